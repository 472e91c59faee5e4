import json, math, numpy as np
from scipy.optimize import least_squares
D=json.load(open('gpurun_out/fit_data.json'))
V={}
for l in open('profiles/r01b/swar_kernel_resources_interior_first.txt'):
    d=dict(kv.split('=') for kv in l.split())
    V[(int(d['ch']),int(d['lw']),int(d['m']),int(d['nw']))]=(int(d['vgpr']),int(d['lds']))
def launch_cycles(p, sh, ch, rb, R, s):
    c_min,c_lat,b_step,b0,fixed,lat_ld = p
    lw,m,nw=sh; np_=lw
    hl=(s*ch+lw-1)//lw
    if 2*hl>=64: return 1e12
    vb=(64-2*hl)*lw
    pairs=(math.ceil(rb/vb)+1)//2
    vrows=m*nw-2*s
    if vrows<=0: return 1e12
    G=pairs*math.ceil(R/vrows)
    vg,lds=V[(ch,lw,m,nw)]
    vw=min(8,512//(((vg+7)//8)*8))
    L=max(1,min(160*1024//lds, vw*4//nw, 32//nw))
    per_cu=math.ceil(G/256)
    rounds=math.ceil(per_cu/L)
    conc=min(per_cu,L)
    k=conc*nw/4.0
    e = (0 if ch == 1 else 2 if ch == 3 else 4) if np_ == 4 else 2 * ch  # lane-crossing taps (folded at np 4)
    stage=(m+2)*(2*np_+e)+m*4*np_+24
    I=s*stage+40+3*m*np_
    rt=I*max(k*c_min,c_lat)+s*b_step+b0+lat_ld*m
    return rounds*rt+fixed
def pred(p,d):
    tot=sum(launch_cycles(p,tuple(d['shape']),d['ch'],d['rb'],R,s) for R,s in d['launches'])
    return tot/d['reps']/2400.0  # us at 2.4 GHz-equivalent cycles
def res(p):
    return np.array([math.log(pred(p,d)/d['us']) for d in D])
p0=[2.8,5.8,300,2000,5000,100]
r=least_squares(res,p0,bounds=([0.5,1,0,0,0,0],[20,50,1e5,1e6,1e6,1e5]))
print("params",np.round(r.x,2))
err=np.exp(np.abs(res(r.x)))
print("median err %.1f%% max %.1f%%"%((np.median(err)-1)*100,(err.max()-1)*100))
print("orig params error:", (np.median(np.exp(np.abs(res(p0))))-1)*100)
# ranking quality: per (src,world,fuse) group, does the model pick a near-best shape?
from collections import defaultdict
g=defaultdict(list)
for d in D: g[(d['src'],d['world'],d['fuse'])].append(d)
tot_loss=0
for k,v in g.items():
    best=min(v,key=lambda d:d['us'])
    pick=min(v,key=lambda d:pred(r.x,d))
    pick0=min(v,key=lambda d:pred(p0,d))
    print(k, "best",best['shape'],best['us'], "| fit pick",pick['shape'],pick['us'], "| old pick", pick0['shape'], pick0['us'])
json.dump(list(r.x),open('gpurun_out/fit_params.json','w'))
