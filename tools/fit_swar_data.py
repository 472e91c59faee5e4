import json, sys, re
sys.path.insert(0, '.')
import pconv
n=pconv.native
V={}
for l in open('profiles/r01b/swar_kernel_resources_interior_first.txt'):
    d=dict(kv.split('=') for kv in l.split())
    V[(int(d['ch']),int(d['lw']),int(d['m']),int(d['nw']))]=(int(d['vgpr']),int(d['lds']))
CH={'grey':1,'rgb':3,'rgba':4}
def load(fn,W,H,reps):
    out=[]
    for l in open(fn):
        if not l.startswith('{'): continue
        r=json.loads(l)
        if r['us_per_rep'] is None or r['shape']=='auto': continue
        world=r['world']; rank=1 if world>1 else 0
        b=n.row_band(H,world,rank)
        halo,fuse=n.normalize_plan(r['halo'],r['fuse'],H//world if world>1 else 0)
        pl=n.plan_band(b,reps,halo,fuse,True,False)
        launches=[(l.hi-l.lo,l.steps) for p in pl for l in p.launches]
        sh=tuple(int(x) for x in r['shape'].split(','))
        ch=CH[r['ch']]
        # shape valid?
        if sh[1]*sh[2]-2*fuse<=0 or 2*((fuse*ch+sh[0]-1)//sh[0])>=64: continue
        out.append(dict(W=W,H=H,ch=ch,rb=W*ch,world=world,reps=reps,fuse=fuse,shape=sh,launches=launches,us=r['us_per_rep'],src=fn.split('/')[-1]))
    return out
# usage: python tools/fit_swar_data.py W:H:REPS:log [...]   (band_sweep.py outputs)
D=[]
for spec in sys.argv[1:]:
    W, H, R, fn = spec.split(':', 3)
    D += load(fn, int(W), int(H), int(R))
json.dump(D,open('gpurun_out/fit_data.json','w'))
print(len(D))
