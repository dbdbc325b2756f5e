"""LDS bank model of the fused CNN's conv1-wgrad B reads (cnn_fused.hip P9).

Lane (lr, lg) of N-tile u reads 4 pixel-pair dwords (2 rows x 2 column pairs) of its tap column kidx = 16 u + lr
from x (kx even), x1 (kx odd, x shifted by one element, its own bank offset X1 from x) or the ones plane (column 25,
offset XONE); lane groups lg 0/1 (and 2/3) share a 32-lane half of each ds_read_b32 access (banks (a/4) mod 32,
one LDS cycle per distinct dword on the busiest bank).  Prints mean cycles per access (1.0 = conflict-free) for
the kernel's placement and sweeps the offsets / cell-pair groupings.
"""
XP=36; NXP=28*36
def make(X1, XONE, junk=17):
    def lane_word(kidx, off):
        if kidx > 25: kidx = junk
        if kidx < 25:
            ky, kx = divmod(kidx, 5)
            if kx & 1: return 100000 + (ky*XP + kx - 1 + off)//2 + X1
            return (ky*XP + kx + off)//2
        return 200000 + off//2 + XONE
    return lane_word
def cost(lw, offs4):
    cyc = 0
    for u in range(2):
        for d in (0, 1, 18, 19):
            for half in (0, 1):
                banks = {}
                for lg in (2*half, 2*half+1):
                    for lr in range(16):
                        w = lw(u*16+lr, offs4[lg]) + d
                        banks.setdefault(w % 32, set()).add(w)
                cyc += max(len(v) for v in banks.values())
    return cyc/16
def off(im, gi):
    py, pc = divmod(gi, 6)
    return im*NXP + py*2*XP + pc*4
def avg(lw, groups): return sum(cost(lw,[off(0,c) for c in g]) for g in groups)/len(groups)
cur=[[k*4+lg for lg in range(4)] for k in range(18)]
print('before (xone at 12, columns 26..31 at x + 0)', avg(make(9,12,junk=26), cur))
print('kernel (xone at 4, columns 26..31 read column 17)', avg(make(9,4), cur))
print('junk->17', avg(make(9,12), cur))
best=[]
for X1 in range(32):
    for XONE in range(32):
        best.append((avg(make(X1,XONE), cur), X1, XONE))
best.sort(); print(best[:6])
r=[]
for XONE in range(32):
    r.append((avg(make(9,XONE), cur), XONE))
print(sorted(r)[:3])
def groups_S(S):
    used=set(); gs=[]
    for j in range(72):
        if j in used: continue
        g=[j+lg*S for lg in range(4)]
        if any(c>=72 or c in used for c in g): return None
        used.update(g); gs.append(g)
    return gs
for S in range(1,19):
    g=groups_S(S)
    if g: print('S',S, min((avg(make(9,XO), g),XO) for XO in range(0,32,4)))
# pair-permuted: lg0=j, lg1=j+T within pairs of k-steps
for T in range(1,40):
    used=set(); gs=[]; ok=True
    for j in range(72):
        if j in used: continue
        # lg0=j, lg1=j+T, lg2=j+1?, lg3=j+1+T
        g=[j, j+T]
        if any(c>=72 or c in used for c in g): ok=False; break
        used.update(g); gs.append(g)
    if not ok: continue
    # combine pairs into k-steps of 4
    ks=[gs[i]+gs[i+1] for i in range(0,len(gs),2)]
    print('T',T, min((avg(make(9,XO), ks),XO) for XO in range(0,32,4)))
