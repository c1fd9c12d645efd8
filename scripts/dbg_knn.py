import sys; sys.path.insert(0,'.'); sys.path.insert(0,'oracle'); sys.path.insert(0,'tests')
import numpy as np, cref
from spatialflink_amd import _abi, synth
from test_gpu_ppoly_ext import agrid, with_edges
ctx=_abi.Context(0)
x,y=synth.uniform(400000,110); off,vx,vy=synth.star_polygons(3,120)
ag,cg=agrid(500)
px,py=vx[off[0]:off[1]],vy[off[0]:off[1]]
wx,wy=with_edges(x,y,np.array([0,len(px)]),px,py)
gi,gd=ctx.knn_ppoly(ag,wx,wy,px,py,0.005,50)
wi,wd=cref.knn_ppoly(cg,wx,wy,px,py,0.005,50)
print("gpu", gi.tolist()); print("orc", wi.tolist())
print("gpu d", gd.tolist()[40:]); print("orc d", wd.tolist()[40:])
print(set(wi.tolist())-set(gi.tolist()), set(gi.tolist())-set(wi.tolist()))
