#!/usr/bin/env python3
"""Exhaustive search of the halo-region chunk swizzle T[p & 15] (conv_wide.hip kHaloSwz):
ds_read_b128 of 16 consecutive pixels (lane fr) x 4 chunks (lane fg), chunk fg ^ T[p] of
128-byte pixel rows, must hit 16 distinct 16-byte bank slots in each of the 4 hardware lane
groups (MI355X_MICROARCH.md LDS table) for every tap start offset."""
import itertools, random, sys
groups = [list(range(0,4))+list(range(12,16))+list(range(20,28)),
          list(range(4,12))+list(range(16,20))+list(range(28,32)),
          list(range(32,36))+list(range(44,48))+list(range(52,60)),
          list(range(36,44))+list(range(48,52))+list(range(60,64))]
def ok(T, offs):
    for o in offs:
        for g in groups:
            seen=set()
            for l in g:
                fr, fg = l & 15, l >> 4
                p = (o + fr)
                slot = ((p & 1) * 8 + (fg ^ T[p & 15])) % 16
                if slot in seen: return False
                seen.add(slot)
    return True
cur = [0,0,1,2,2,0,4,4,5,5,6,2,2,6,6,7]
print("current ok for {15,0,1}:", ok(cur,[15,0,1]), " all16:", ok(cur, range(16)))
need = [0,1,2,4,6,10,12,14,15]
print("current ok for need:", ok(cur, need))
# backtracking search
def search(offs):
    T=[None]*16
    order=list(range(16))
    def partial_ok(k):
        # check constraints only involving assigned entries
        for o in offs:
            for g in groups:
                seen=set()
                for l in g:
                    fr, fg = l & 15, l >> 4
                    p=(o+fr)&15
                    if T[p] is None: continue
                    slot=((p&1)*8 + (fg ^ T[p]))%16
                    if slot in seen: return False
                    seen.add(slot)
        return True
    def rec(k):
        if k==16: return True
        for v in range(8):
            T[k]=v
            if partial_ok(k) and rec(k+1): return True
        T[k]=None
        return False
    return T if rec(0) else None
for offs in [list(range(16)), need]:
    r=search(offs); print(offs, r)
