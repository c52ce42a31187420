"""NumPy model of K3's phase-A screens on the bench's own maps (round 4): the fraction of cells each
screen passes to the candidate test, for the round-3 pair screen, mean-offset levels and quantile
levels (cfar2d.hpp FMCW_K3_LV_QA / _QB), against the exact E(s_min) >= need test.  The maps are the
bench's synthetic frames (seed 1234) through the C restatement (oracle/fmcw_cpu.c); rows sampled at
5 positions, 48 CUT rows each.  usage: python tools/k3_screen_model.py"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "fpga-fmcw-radar-processor_amd"))
sys.path.insert(0, str(REPO / "oracle"))


def bench_maps():
    import cpu_backend as CB
    from fmcw import synth
    out = {}
    for name, (ns, nc, nrx, dt) in {"c5": (8192, 1024, 1, "f16"), "c3": (4096, 512, 4, "f32"),
                                    "c2": (1024, 256, 1, "f32")}.items():
        cube = synth.frames(1, ns, nc, nrx, "two_targets", seed=1234, dtype=dt)
        if not np.iscomplexobj(cube):
            x = cube.astype(np.float32)
            cube = x[..., 0] + 1j * x[..., 1]
        m, _, _ = CB.process(cube.astype(np.complex64), None, threads=8)
        out[name] = m[0]
    return out


Z = bench_maps()
hr,gr,hd,gd=5,1,6,2
offs=[(dr,dd) for dr in range(-hr,hr+1) for dd in range(-hd,hd+1) if not (abs(dr)<=gr and abs(dd)<=gd)]
need=32; s=np.float32(2.0)
def k16(v): return (np.asarray(v,np.float32).view(np.uint32)>>16).astype(np.int64)
def lo(k): return (np.asarray(k,np.uint32)<<16).view(np.float32)
def levels_mean(first, dA=56, dB=80):
    M=int(((first.view(np.uint32)>>19).astype(np.int64)).mean())*8
    return [M+dA, M+dB]
def levels_q(first, pa, pb):
    k7=(first.view(np.uint32)>>19).astype(np.int64).ravel()
    return [int(np.quantile(k7,pa))*8, int(np.quantile(k7,pb))*8]
def evalchunk(m, r0, nrows, Qs):
    R=m[r0-hr:r0+nrows+hr]
    cut=R[hr:-hr]
    refs=np.stack([np.roll(R,(-dr,-dd),axis=(0,1))[hr:-hr] for dr,dd in offs],-1)
    E=((s*refs)>=cut[...,None]).sum(-1)
    rk=k16(refs); ck=k16(cut)
    res={"exact":(E<need).mean()}
    pm=np.maximum(R,np.roll(R,-1,axis=1))
    pairs=[(dr,p) for dr in range(-hr,hr+1) for p in ([-6,-4,3,5] if abs(dr)<=gr else [-6,-4,-2,0,2,4])]
    pv=np.stack([np.roll(pm,(-dr,-dd),axis=(0,1))[hr:-hr] for dr,dd in pairs],-1)
    res["pair"]=((s*pv>=cut[...,None]).sum(-1)<need).mean()
    for name,Q in Qs.items():
        surv=np.ones(cut.shape,bool)
        for q in Q:
            q=max(1,min(q,0x7f80)); U=int(k16(s*lo(q)))
            surv&=~((ck<U)&((rk>=q).sum(-1)>=need))
        res[name]=surv.mean()
    return res
for name in ("c5","c3","c2"):
    m=Z[name]; ns=m.shape[0]
    acc={}
    for r0 in [20, ns//8, ns//4+7, ns//2, 3*ns//4-20]:
        first=m[r0:r0+4]
        Qs={"mean56_80":levels_mean(first)}
        for pa,pb in [(0.60,0.70),(0.55,0.65),(0.5,0.62),(0.56,0.68),(0.58,0.66),(0.52,0.68)]:
            Qs[f"q{pa}_{pb}"]=levels_q(first,pa,pb)
        k7=(first.view(np.uint32)>>19).astype(np.int64).ravel()
        Qs["4lv"]=[int(np.quantile(k7,p))*8 for p in (0.5,0.58,0.66,0.74)]
        Qs["3lv"]=[int(np.quantile(k7,p))*8 for p in (0.52,0.62,0.72)]
        r=evalchunk(m, r0, 48, Qs)
        for k,v in r.items(): acc.setdefault(k,[]).append(v)
    print(name, {k: "%.3f%%"%(100*np.mean(v)) for k,v in acc.items()})
