import numpy as np
p=21888242871839275222246405745257275088696311157297823662689037894645226208583
d=np.fromfile('mul29_check.bin',dtype=np.uint32).reshape(3,-1,9)
R=2**261; Ri=pow(R,-1,p)
def val(l): return sum(int(x)<<(29*i) for i,x in enumerate(l))
bad=0
for a,b,o in zip(*d):
    A,B,O=val(a),val(b),val(o)
    if O%p != A*B*Ri%p or O >= 2*p: bad+=1
print('mul29 mismatches:',bad,'of',d.shape[1])
