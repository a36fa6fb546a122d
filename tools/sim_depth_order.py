# Wave-maximum cost model of ordering a tile of sites by depth before the main kernel
# scores it 64 at a time: key-build chunks and big fold-chain
# steps per 64-site block at Poisson(60) / Poisson(30) depths, unsorted vs sorted tiles.
import numpy as np
rng=np.random.default_rng(1)
N=1<<22
nt=rng.poisson(60,N); nn=rng.poisson(30,N)
def cost(nt,nn):
    nt=nt.reshape(-1,64); nn=nn.reshape(-1,64)
    nt4=(nt+3)//4*4
    joint=(nt4+nn<=128).all(1)
    ch=np.where(joint,((nt4+nn+3)//4).max(1),(nt4//4).max(1)+((nn+3)//4).max(1))
    ft=np.ceil(nt.max(1)/4); fn=np.ceil(nn.max(1)/4)
    passes=np.where(joint,1,2)
    return dict(chunks=ch.mean(), fold=(ft+fn).mean(), sep=(~joint).mean(), net=passes.mean())
base=cost(nt,nn); print('unsorted',base)
for W in (128,256,512,1024):
    for name,key in (('nt+nn',nt+nn),('2nt+nn',2*nt+nn),('nt',nt),('nt4+nn',(nt+3)//4*4+nn)):
        k=key.reshape(-1,W); idx=np.argsort(k,axis=1,kind='stable')
        o=(idx+np.arange(0,N,W)[:,None]).ravel()
        c=cost(nt[o],nn[o]); print(W,name,{k:round(v,3) for k,v in c.items()})
print('mean chunks',((nt+3)//4*4+nn).mean()/4,'mean fold',(nt/4+nn/4).mean())
print('2D')
for W in (256,512):
    for A in (2,4):
        k1=nt.reshape(-1,W); i1=np.argsort(k1,axis=1,kind='stable')
        o=(i1+np.arange(0,N,W)[:,None])   # rows sorted by nt
        # split into A classes, sort each by nn
        o=o.reshape(-1,W//A)
        k2=nn[o]; i2=np.argsort(k2,axis=1,kind='stable')
        o2=np.take_along_axis(o,i2,1).ravel()
        c=cost(nt[o2],nn[o2]); print(W,A,{k:round(v,3) for k,v in c.items()})
