import sys, os
sys.path.insert(0,'oracle'); sys.path.insert(0,'gnark-icicle_amd')
os.environ['GM_DEBUG_MSM']='1'
import pyref, gnark_mi355x as gm
ctx=gm.Context(0)
for cname in ['bn254','bls12377']:
  c=pyref.CURVES[cname]
  for g2 in [False,True]:
    P0=pyref.random_points(c,1,5,g2)[0]
    S=ctx.copy_to_device(pyref.encode_fr(c,12345))
    P=ctx.copy_points_to_device(cname,pyref.encode_point(c,P0,g2),g2)
    jac,aff=ctx.msm(cname,S,P,1,g2)
    print(cname,g2,pyref.decode_point(c,aff,g2)==pyref.Group(c,g2).mul(P0,12345), jac.hex()[:64], flush=True)
