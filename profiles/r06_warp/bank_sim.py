import numpy as np
rng=np.random.default_rng(1)
def cost(P, layout, nbank=32):
    tot=0; cnt=0
    for th in np.arange(0,360,3.0):
        c,s=np.cos(np.radians(th)),np.sin(np.radians(th))
        for trial in range(4):
            ox,oy=rng.uniform(8,16),rng.uniform(8,16)
            for i in range(4):
                for u in range(4):
                    for half in range(2):
                        if layout=='A':
                            lr=np.arange(4)+4*half; lg=np.arange(8)
                            LR,LG=np.meshgrid(lr,lg,indexing='ij'); x=4*LG+u; y=LR+8*i
                        elif layout=='B':
                            lr=np.arange(4)+4*half; lg=np.arange(8)
                            LR,LG=np.meshgrid(lr,lg,indexing='ij'); x=LG+8*u; y=LR+8*i
                        else:  # row of 32
                            x=np.arange(32); y=np.full(32, 8*u+4*half+i)
                        sx=np.floor(x*c-y*s+ox+20).astype(int); sy=np.floor(x*s+y*c+oy+20).astype(int)
                        for tap in [(0,0),(1,0),(0,1),(1,1)]:
                            a=(sy+tap[1])*P+(sx+tap[0])
                            d=np.unique((a//4).ravel())
                            m=np.bincount(d%nbank).max()
                            tot+=m; cnt+=1
    return tot/cnt
for lay in 'ABC':
    for P in [68,72,76]:
        print(lay, P, round(cost(P,lay),3))
