"""Bank-conflict model of the LDS FFT passes (fft_device.hpp FftPlan).

A ds_read/ds_write_b128 serves 16 lanes per cycle when their 16-B slots
(index mod 16 of the double2 LDS image) are distinct; the degree of a 16-lane
group is the largest number of lanes on one slot.  Prints the mean degree
(1.0 = conflict-free) of every pass store/load of a plan, for the old padded
layout (i + i/16) and the XOR swizzle lds_slot().

  python3 tools/lds_conflicts.py
"""


def plan(M, V):
    LOG, LOGV = M.bit_length() - 1, V.bit_length() - 1
    NP = (LOG + LOGV - 1) // LOGV
    R0 = 1 << (LOG - LOGV * (NP - 1))
    return NP, R0, M // V


def accesses(M, V):
    NP, R0, T = plan(M, V)
    radix = lambda p: R0 if p == 0 else V
    ns = lambda p: 1 if p == 0 else R0 * (1 << ((V.bit_length() - 1) * (p - 1)))
    acc = []
    for p in range(NP - 1):
        R, NS = radix(p), ns(p)
        for b in range(V // R):
            for r in range(R):
                acc.append([((t + b * T) // NS) * NS * R + ((t + b * T) & (NS - 1)) + r * NS for t in range(T)])
        R1 = radix(p + 1)
        for b in range(V // R1):
            for r in range(R1):
                acc.append([t + b * T + r * (M // R1) for t in range(T)])
    return acc


def degree(acc, f):
    tot = n = 0
    for addrs in acc:
        for g in range(0, len(addrs), 16):
            slots = [f(a) % 16 for a in addrs[g:g + 16]]
            tot += max(slots.count(s) for s in set(slots))
            n += 1
    return tot / n


def pad(i):
    return i + i // 16


def lds_slot(i):
    q = i >> 4
    return i ^ ((q ^ ((q & 4) << 1)) & 15)


if __name__ == "__main__":
    for M, V in [(4096, 8), (2048, 8), (1024, 8), (1024, 16), (512, 16), (256, 16)]:
        acc = accesses(M, V)
        print(f"M={M:5d} V={V:2d} passes/R0/T={plan(M, V)}  pad {degree(acc, pad):.3f}  "
              f"lds_slot {degree(acc, lds_slot):.3f}")
