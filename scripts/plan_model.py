"""Host-side model of the grouped forward projector's angle-group planner (admm_tomo.hip,
admm_ctx_create: plan_group / the greedy loop) for sweeping its parameters without a GPU.
usage: python scripts/plan_model.py N ANGLES SEGMENTS GMAX WIN RAYS [FULL_ANGLES]
Prints, for the unaligned and the ray-aligned plan: group sizes, blocks, touched row pixels
per launch (staged_px) and pixels fetched by the 64-slot LDS-DMA pieces (fetched_px; MB at
32 B per pixel = 8 float32 nodes)."""
import math, sys
N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
NA = int(sys.argv[2]) if len(sys.argv) > 2 else 96
SEG = int(sys.argv[3]) if len(sys.argv) > 3 else 8
GMAX = int(sys.argv[4]) if len(sys.argv) > 4 else 16
WIN = int(sys.argv[5]) if len(sys.argv) > 5 else 256
RAYS = int(sys.argv[6]) if len(sys.argv) > 6 else 64
NFULL = int(sys.argv[7]) if len(sys.argv) > 7 else NA  # angle step pi/NFULL (mirror half: NA = NFULL/2)
ndet = N
h = 2.0 / N; hd = 2.0 / ndet; c0 = 0.5 * (N - 1); det_min = -1.0
fa = []
for t in range(NA):
    th = (t + 0.5) * math.pi / NFULL
    cs, sn = math.cos(th), math.sin(th)
    caseA = abs(cs) >= abs(sn)
    al, be = (cs, sn) if caseA else (sn, cs)
    fa.append(dict(A0=c0 + (det_min / h + 0.5 * hd / h + c0 * be) / al, A1=(hd / h) / al, dl=-be / al, caseA=caseA))
cd = 0.5 * (ndet - 1)

def plan_group(t0, G, align):
    if any(fa[t0 + q]['caseA'] != fa[t0]['caseA'] for q in range(G)):
        return None
    blocks = 0; staged = 0; fetched = 0
    for s in range(SEG):
        mlo, mhi = s * N // SEG, (s + 1) * N // SEG
        mc = 0.5 * (mlo + mhi - 1)
        r0 = fa[t0]
        lref = r0['A0'] + cd * r0['A1'] + mc * r0['dl']
        ds = []
        for q in range(G):
            b = fa[t0 + q]
            d = round((lref - b['A0'] - cd * b['A1'] - mc * b['dl']) / b['A1']) if align else 0
            ds.append(d)
        kcb = math.floor(-max(ds) / RAYS); kce = math.ceil((ndet - min(ds)) / RAYS)
        for kc in range(kcb, kce):
            blocks += 1
            for m in range(mlo, mhi):
                lo, hi = 1e300, -1e300
                for q in range(G):
                    b = fa[t0 + q]
                    ka = max(kc * RAYS + ds[q], 0); kb = min(kc * RAYS + ds[q] + RAYS - 1, ndet - 1)
                    if ka > kb: continue
                    for kk in (ka, kb):
                        l = m * b['dl'] + (kk * b['A1'] + b['A0'])
                        lo = min(lo, l); hi = max(hi, l)
                if lo > hi: continue
                w = math.floor(hi) - math.floor(lo) + 2
                if w > WIN - 2: return None
                staged += w
                fetched += sum(1 for hh in range((WIN // 2 + 63) // 64) for par in (0, 1) if 128 * hh + par < w + 1) * 64
    return blocks, staged, fetched

for align in (False, True):
    t0 = 0; Gs = []; B = S = F = 0
    while t0 < NA:
        G = min(GMAX, NA - t0)
        while G > 1 and plan_group(t0, G, align) is None: G -= 1
        r = plan_group(t0, G, align)
        Gs.append(G); B += r[0]; S += r[1]; F += r[2]; t0 += G
    print(f"align={align} groups={Gs} blocks={B} staged_px={S/1e6:.2f}M fetched_px={F/1e6:.2f}M fetchedMB={F*32/1e6:.0f}")
