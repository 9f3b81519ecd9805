"""CPU measurement (DESIGN.md §8.3 hypothesis): do numpy-legacy Fisher-Yates
walks (permutation(n) = n-1 masked-rejection draws on MT19937, the stream the
target creators' np.random.choice consumes) started from neighbouring stream
offsets coalesce before the call ends?  Prints, for calls of n elements, the
number of distinct end offsets over consecutive candidate starts, and how the
number of distinct walk states shrinks along a 12,000-element call.

    python tools/probe_coalesce.py
"""
import numpy as np
raw = np.random.MT19937(12345).random_raw(2_000_000).astype(np.uint64)
def mask_of(i):
    m = i; m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16
    return m
def walk_end(starts, n):
    pos = starts.copy()
    for i in range(n - 1, 0, -1):
        m = mask_of(i)
        act = np.ones(len(pos), bool)
        while act.any():
            u = raw[pos[act]] & m
            ok = u <= i
            idx = np.nonzero(act)[0]
            pos[idx] += 1
            act[idx[ok]] = False
    return pos
for n in [50, 200, 1000, 5000, 12000]:
    s0 = 1000
    starts = np.arange(s0, s0 + 64, dtype=np.int64)
    e = walk_end(starts, n)
    print(n, 'distinct ends over 64 consecutive starts:', len(np.unique(e)), ' draws ~', e[0]-starts[0])
# wider start ranges and merge time
def walk_trace(starts, n, every=500):
    pos = starts.copy(); out=[]
    for k, i in enumerate(range(n - 1, 0, -1)):
        m = mask_of(i)
        act = np.ones(len(pos), bool)
        while act.any():
            u = raw[pos[act]] & m
            ok = u <= i
            idx = np.nonzero(act)[0]
            pos[idx] += 1
            act[idx[ok]] = False
        if k % every == 0 or k < 64 and k % 8 == 0: out.append((k, len(np.unique(pos))))
    return pos, out
starts = np.arange(5000, 7000, dtype=np.int64)
e, tr = walk_trace(starts, 12000)
print('2000 starts, n=12000: distinct ends', len(np.unique(e)))
print('distinct states after k steps:', tr[:20])
