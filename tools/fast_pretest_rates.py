# Pass rates of the FAST compass pre-test and of the full segment test on a synthetic
# KITTI-size frame (numpy; evidence for the FAST tile-height decision in DESIGN.md section 5).
import sys, numpy as np
sys.path.insert(0, '/root/repo')
from svo_amd.scene import Scene
sc = Scene(1241, 376, seed=101)
img = sc.frame(3).astype(np.int32)
H, W = img.shape
ring = [(0,3),(1,3),(2,2),(3,1),(3,0),(3,-1),(2,-2),(1,-3),(0,-3),(-1,-3),(-2,-2),(-3,-1),(-3,0),(-3,1),(-2,2),(-1,3)]
v = img[3:H-3, 3:W-3]; t = 20
R = np.stack([img[3+dy:H-3+dy, 3+dx:W-3+dx] for dx, dy in ring])
br = R > v + t; dk = R < v - t
def comp(m): return (m[0] | m[8]) & (m[4] | m[12])
cand = comp(br) | comp(dk)
def runk(m, idx, k):
    s = m[idx]; n = len(idx); out = np.zeros(s.shape[1:], bool)
    for st in range(n):
        a = np.ones(s.shape[1:], bool)
        for j in range(k): a &= s[(st + j) % n]
        out |= a
    return out
ev = list(range(0, 16, 2))
cand2 = runk(br, ev, 4) | runk(dk, ev, 4)
corner = runk(br, list(range(16)), 9) | runk(dk, list(range(16)), 9)
N = v.size
print(f"compass {cand.mean():.4f}  evens-run4 {cand2.mean():.4f}  corner {corner.mean():.4f}  (both {(cand & cand2).mean():.4f})")
