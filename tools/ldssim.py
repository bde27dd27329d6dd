"""LDS bank-conflict model of the D = 4 FIR wave (fir_poly_kernel) (tuning aid):
every ds op of the wave as 8-byte accesses in 4 groups of 16 lanes, bank =
dword mod 32, extra cycles = the busiest bank's distinct dwords - 1 per group
(MI355X_MICROARCH.md LDS table).  The model gives 96 extra cycles per wave for
round 2's layout, exactly SQ_LDS_BANK_CONFLICT / waves of the PMC pass
(pmc_c5_r02_v38.json: 134.2 M / 1.398 M waves); all of it in Plan256d's
second exchange, which xpad<Plan256d, 2> (fft_engine.hpp) removes; likewise
256 per D = 1 FIR wave (Plan1024x, pmc_c2_r02_v38.json: 44.6 M / 174,309 waves),
removed by xpad<Plan1024x, 2>.
  python tools/ldssim.py"""
import itertools

def conflicts(addrs_f2):       # list of 64 float2 indices (or None for inactive)
    extra = 0
    for g in range(4):
        banks = {}
        for l in range(16 * g, 16 * g + 16):
            a = addrs_f2[l]
            if a is None: continue
            for dw in (2 * a, 2 * a + 1):
                banks.setdefault(dw % 32, set()).add(dw)
        extra += max(len(v) for v in banks.values()) - 1 if banks else 0
    return extra

def pair_map(t): return ((t & 31) << 1) | (t >> 5)

def run(PADSH_F=5, PADUN_F=0, PADSH_I=4, PADUN_I=0, tqmap=lambda t: (t & 15) | ((t & 16) << 1) | ((t & 32) >> 1), verbose=False):
    padF = lambda i: (i >> PADSH_F) << PADUN_F
    padI = lambda i: (i >> PADSH_I) << PADUN_I
    tot = 0; ninst = 0
    # front Plan1024q: N=1024, E=16, R=[16,16], TF=64. pass0 store: j = pair(t), Ns=1: out r at 16 j + r
    for r in range(16):
        addrs = [16 * pair_map(t) + r + padF(16 * pair_map(t) + r) for t in range(64)]
        tot += 2 * conflicts(addrs); ninst += 2   # a and d
    # pass1 load (id map): v[r] = lds[t + 64 r]
    for r in range(16):
        addrs = [t + 64 * r + padF(t + 64 * r) for t in range(64)]
        tot += 2 * conflicts(addrs); ninst += 2
    # inverse Plan256d: N=256, E=4, R=[4,4,4,4], TF=64, thread tq
    Ns = 1
    for p in range(4):
        R = 4
        if p < 3:   # store pass p output
            for r in range(R):
                addrs = []
                for t in range(64):
                    j = tqmap(t)
                    hi = (j // Ns) * Ns * R
                    i = hi + (j % Ns) + r * Ns
                    addrs.append(i + padI(i))
                c = conflicts(addrs)
                if verbose: print("inv store p", p, "r", r, c)
                tot += 2 * c; ninst += 2
        if p > 0:   # load pass p input: v[r] = lds[j + r N/R]
            for r in range(R):
                addrs = []
                for t in range(64):
                    j = tqmap(t)
                    i = j + r * 64
                    addrs.append(i + padI(i))
                c = conflicts(addrs)
                if verbose: print("inv load p", p, "r", r, c)
                tot += 2 * c; ninst += 2
        Ns *= R
    return tot, ninst


def plan1024x(x1, x2):
    """One transform of the D = 1 FIR's Plan1024x (radices 16, 4, 16; pair
    lane map in the first and last pass): extra LDS cycles with exchange 1
    padded (S1, U1) and exchange 2 (S2, U2)."""
    (S1, U1), (S2, U2) = x1, x2
    p1 = lambda i: i + ((i >> S1) << U1)
    p2 = lambda i: i + ((i >> S2) << U2)
    tot = sum(conflicts([p1(16 * pair_map(t) + r) for t in range(64)]) for r in range(16))
    tot += sum(conflicts([p1(t + 64 * b + 256 * r) for t in range(64)]) for b in range(4) for r in range(4))
    tot += sum(conflicts([p2((t + 64 * b) // 16 * 64 + (t + 64 * b) % 16 + 16 * r) for t in range(64)])
               for b in range(4) for r in range(4))
    tot += sum(conflicts([p2(pair_map(t) + 64 * r) for t in range(64)]) for r in range(16))
    return tot



def conf_groups(addr_dw, groups, nbanks, width):
    """Extra cycles of one ds op: per lane group, the busiest bank's distinct
    dwords - 1 (addr_dw: first dword per lane, width dwords per lane)."""
    extra = 0
    for g in groups:
        banks = {}
        for l in g:
            for k in range(width):
                dw = addr_dw[l] + k
                banks.setdefault(dw % nbanks, set()).add(dw)
        extra += max(len(v) for v in banks.values()) - 1
    return extra


G8 = [list(range(8 * g, 8 * g + 8)) for g in range(8)]            # ds_write_b128
G16 = [list(range(16 * g, 16 * g + 16)) for g in range(4)]         # ds_write_b64
G32 = [list(range(32)), list(range(32, 64))]                       # ds_read_b64
GR128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
         [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
GR128 += [[l + 32 for l in g] for g in GR128]                     # ds_read_b128


def psd8192i(x1, x2, wave=0):
    """One frame of the PSD's Plan8192i (radices 16, 32, 16; interleaved first
    and last pass) for wave `wave` of the 256-thread block: extra LDS cycles."""
    (S1, U1), (S2, U2) = x1, x2
    p1 = lambda i: i + ((i >> S1) << U1)
    p2 = lambda i: i + ((i >> S2) << U2)
    T = [64 * wave + l for l in range(64)]
    tot = sum(conf_groups([2 * p1(32 * t + 16 * b + r) for t in T], G8, 32, 4)
              for b in range(2) for r in range(0, 16, 2))
    tot += sum(conf_groups([2 * p1(t + 256 * r) for t in T], G32, 64, 2) for r in range(32))
    tot += sum(conf_groups([2 * p2((t // 16) * 512 + t % 16 + 16 * r) for t in T], G16, 32, 2)
               for r in range(32))
    tot += sum(conf_groups([2 * p2(2 * t + 512 * r) for t in T], GR128, 64, 4) for r in range(16))
    return tot


def run_x(xpads, tqmap):
    tot = 0
    Ns = 1
    for p in range(4):
        if p < 3:
            S, U = xpads[p + 1]
            for r in range(4):
                addrs = []
                for t in range(64):
                    j = tqmap(t); hi = (j // Ns) * Ns * 4; i = hi + (j % Ns) + r * Ns
                    addrs.append(i + ((i >> S) << U))
                tot += conflicts(addrs)
        if p > 0:
            S, U = xpads[p]
            for r in range(4):
                addrs = []
                for t in range(64):
                    j = tqmap(t); i = j + r * 64
                    addrs.append(i + ((i >> S) << U))
                tot += conflicts(addrs)
        Ns *= 4
    return 2 * tot
tq = lambda t: (t & 15) | ((t & 16) << 1) | ((t & 32) >> 1)
idm = lambda t: t
if __name__ == "__main__":
    print("fir_poly_kernel wave, front + inverse (extra LDS cycles, LDS instructions):", run())
    for name, m in (("poly (lanes tq)", tq), ("dec (lanes t)", idm)):
        print(f"Plan256d inverse, {name}: 1 pad / 16 everywhere", run_x({1: (4, 0), 2: (4, 0), 3: (4, 0)}, m),
              "| exchange 2 with 4 pads / 16", run_x({1: (4, 0), 2: (4, 2), 3: (4, 0)}, m))
    # fir_os_kernel<Plan1024x>: 4 transforms per wave (2 segments, forward + inverse)
    print("D = 1 FIR wave (Plan1024x): 1 pad / 32 everywhere", 4 * plan1024x((5, 0), (5, 0)),
          "| exchange 2 with 1 pad / 16", 4 * plan1024x((5, 0), (4, 0)))
    print("PSD frame, waves 0-3 (Plan8192i): 2 pads / 32 everywhere",
          [psd8192i((5, 1), (5, 1), w) for w in range(4)],
          "| exchange 2 with 2 pads / 64", [psd8192i((5, 1), (6, 1), w) for w in range(4)])
