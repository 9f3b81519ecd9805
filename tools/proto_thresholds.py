"""CPU check of the threshold form of a chunk of numpy's masked-rejection draws
(the chip-wide sampler's chunk functions), before any kernel is written.

Within one mask region (steps i in [lo, hi], mask hi = 2^b - 1, lo = 2^(b-1))
word t of a chunk is accepted iff the step it meets is >= v_t = w_t & hi.  The
step it meets is i_in - (accepted before t), so acceptance is monotone in the
entering step i_in: word t is accepted iff i_in >= tau_t, with
    tau_t = v_t + #{s < t : u_s <= v_t},
where u_s = tau_s - rank(tau_s) is kept per inserted threshold and every
u_s > v_t drops by one at the insertion of v_t.  So the chunk's function for
every i_in of the region is 64 integers: accepted = ballot(tau <= i_in).
A path that leaves the region inside the chunk (crosses lo) continues from the
exact step lo - 1 at the word after its (i_in - lo + 1)-th acceptance; that
suffix is a function of the word index alone (a 64-entry crossing table).

    python tools/proto_thresholds.py
"""
import numpy as np


def mask_for(i):
    return (1 << int(i).bit_length()) - 1


def serial(words, i, lo_stop=1):
    """Walk words from step i (one call, no end); returns accepted flags."""
    acc = []
    for w in words:
        v = int(w) & mask_for(i)
        a = i >= 1 and v <= i
        acc.append(a)
        if a:
            i -= 1
    return acc, i


def thresholds(words, hi):
    u, tau = [], []
    for w in words:
        v = int(w) & hi
        k = sum(1 for x in u if x <= v)
        tau.append(v + k)
        u = [x - 1 if x > v else x for x in u]
        u.append(v)
    return tau


def check(seed, b, L=64, trials=None):
    rng = np.random.default_rng(seed)
    hi, lo = (1 << b) - 1, 1 << (b - 1)
    words = rng.integers(0, 1 << 32, size=L, dtype=np.uint64)
    tau = thresholds(words, hi)
    cross = {}  # t* -> (accepted flags of the suffix, exit step)
    for ts in range(L + 1):
        cross[ts] = serial(words[ts:], lo - 1)
    bad = 0
    for i_in in range(lo, hi + 1):
        ref, i_out = serial(words, i_in)
        acc = [tau[t] <= i_in for t in range(L)]
        n_before_last = sum(acc[:-1])
        if n_before_last <= i_in - lo:           # the path stays in the region
            got, g_out = acc, i_in - sum(acc)
        else:                                    # crossing: t* after the (i_in-lo+1)-th acceptance
            need = i_in - lo + 1
            cnt, ts = 0, None
            for t in range(L):
                cnt += acc[t]
                if acc[t] and cnt == need:
                    ts = t + 1
                    break
            sfx, g_out = cross[ts]
            got = acc[:ts] + sfx
        if got != ref or g_out != i_out:
            bad += 1
    return bad, hi - lo + 1


if __name__ == "__main__":
    tot = 0
    for b in (2, 3, 5, 6, 7, 8, 10, 13):
        for seed in range(6 if b < 12 else 2):
            bad, n = check(seed * 31 + b, b)
            tot += bad
            print(f"mask {(1 << b) - 1:5d} seed {seed}: {n} entering steps, {bad} mismatches")
    print("total mismatches", tot)
