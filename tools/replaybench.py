import sys, time, numpy as np
sys.path.insert(0,'/root/repo'); import pkgload; pkgload.load()
from theta_rrt_amd import _native as N
rng=np.random.default_rng(0)
B=4096
b=N.Book(); b.reset([16.0,16.0,0.0]); ts=[]
for step in range(40):
    n=b.size()
    rs=np.zeros(B,N.RESOLVED_DTYPE)
    ok=rng.random(B)<0.6
    rs['r']['status']=np.where(ok, N.ST_OK, N.ST_COLLISION)
    rs['r']['near']=rng.integers(0,n,B)
    dup=ok & (rng.random(B)<0.25)
    first=ok & ~dup
    nf=int(first.sum())
    rs['idx']=-1
    rs['idx'][first]=n+np.arange(nf)
    rs['idx'][dup]=rng.integers(0,n,int(dup.sum()))
    rs['flags'][first]=N.RS_FIRST
    t=time.perf_counter(); b.replay(rs); ts.append(time.perf_counter()-t)
print("nodes",b.size(),"replay us last5",[round(x*1e6) for x in ts[-5:]])
for dupfrac, okfrac in ((0.0,0.6),(0.25,0.6),(0.0,0.0),(0.0,1.0)):
    b=N.Book(); b.reset([16.0,16.0,0.0]); b.reserve(200000,200000); ts=[]
    for step in range(30):
        n=b.size()
        rs=np.zeros(B,N.RESOLVED_DTYPE)
        ok=rng.random(B)<okfrac
        rs['r']['status']=np.where(ok, N.ST_OK, N.ST_COLLISION)
        rs['r']['near']=rng.integers(0,n,B)
        dup=ok & (rng.random(B)<dupfrac); first=ok & ~dup; nf=int(first.sum())
        rs['idx']=-1; rs['idx'][first]=n+np.arange(nf); rs['idx'][dup]=rng.integers(0,n,int(dup.sum()))
        rs['flags'][first]=N.RS_FIRST
        t=time.perf_counter(); b.replay(rs); ts.append(time.perf_counter()-t)
    print(dupfrac, okfrac, "nodes",b.size(),[round(x*1e6) for x in ts[-4:]])
