import sys; sys.path[:0]=['linear-program-solver_amd','.']
from lpsol_amd import _lib
from lpsol_amd import generators as gen
_lib.load()
for (kind,m,ns) in [("mixed",9000,3000),("tall",20000,200),("tall",32768,40),("tall",32768,8192)]:
    T=gen.tableau(kind,m,ns,1)
    for b in (48,64):
        e=_lib.Engine(T.shape[0]-1,T.shape[1]-1); e.upload(T); e.set_block(b)
        print(kind,m,ns,b,e.geometry(),flush=True); e.close()
