"""Host dry run of tests/test_gpu_lm_stress.py's gate (the host build of the register path in place of
the GPU): candidates beyond 5e-10 of the C port, refitted by the numpy oracle, classified by the
oracle's own one-ulp spread; detail() prints the unexplained ones. Measured r05: ndata 5 / 10 / 16
beyond the resolution 32 / 4 / 5, unexplained 10 / 2 / 2 (6.2e-5 / 1.4e-5 / 1.4e-5 of status 0)."""
import sys, os, ctypes, numpy as np, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'tests', 'helpers'))
from test_gpu_lm_stress import _vectors
from conftest import wrapped
import lm_oracle_check as LC
import multiprocessing as mp
from concurrent.futures import ProcessPoolExecutor
P=ctypes.c_void_p
hc = ctypes.CDLL(os.path.join(ROOT, 'tests', 'hostcheck', 'libhostcheck.so'))
hc.hc_fit_segments.argtypes = [P, ctypes.c_long, ctypes.c_int, P, P, P, ctypes.c_int, P, P, P, ctypes.c_int]
cl = ctypes.CDLL(os.path.join(ROOT, 'oracle', 'libnls_scalar.so')); cl.lm_scalar_fit.argtypes = [P, ctypes.c_int64, ctypes.c_int, P, ctypes.c_int, P]
CONSTS = np.array([100, 1e-9, 1e-9, 1e-3, 5.0, 30.0, 0.5, 0.05, 0.1, 1e-15]); LAMS = np.array([0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0])
def main():
    for nd in (5,10,16):
        n=200000; qi,guess=_vectors(nd,n,1000+nd)
        ref=np.zeros((n,6)); cl.lm_scalar_fit(qi.ctypes.data,n,nd,guess.ctypes.data,8,ref.ctypes.data)
        qcm=np.ascontiguousarray(qi.T); gp=np.zeros((n,4)); ss=np.zeros(n); gs=np.zeros(n,np.int32)
        hc.hc_fit_segments(qcm.ctypes.data,n,nd,guess.ctypes.data,CONSTS.ctypes.data,LAMS.ctypes.data,8,gp.ctypes.data,ss.ctypes.data,gs.ctypes.data,0)
        rs=ref[:,5].astype(int); match=gs==rs; both0=match&(rs==0)
        d=np.stack([np.abs(gp[:,0]-ref[:,0]),np.abs(gp[:,1]-ref[:,1]),wrapped(gp[:,2]-ref[:,2]),np.abs(gp[:,3]-ref[:,3])],axis=1)
        cand=np.nonzero(both0&(d.max(1)>5e-10))[0]
        t0=time.time()
        with ProcessPoolExecutor(8, mp_context=mp.get_context("spawn")) as ex:
            orc=list(ex.map(LC.oracle_fit,[(nd,qi[k],guess[k]) for k in cand],chunksize=32))
            beyond=[(k,o) for k,o in zip(cand,orc) if o[0]==0 and np.any(LC._dist(gp[k][None],o[1][None])[0]>o[2])]
            spreads=list(ex.map(LC.oracle_spread,[(nd,qi[k],guess[k],o[1],4) for k,o in beyond]))
        un=[int(k) for (k,o),sp in zip(beyond,spreads) if np.any(LC._dist(gp[k][None],o[1][None])[0]>np.maximum(o[2],1.5*sp))]
        print(nd,'match',match.mean(),'cand',cand.size,'beyond',len(beyond),'unexplained',len(un),un[:5],'oracle s',round(time.time()-t0,1))

def detail():
    nd=5; n=200000; qi,guess=_vectors(nd,n,1005)
    qcm=np.ascontiguousarray(qi.T); gp=np.zeros((n,4)); ss=np.zeros(n); gs=np.zeros(n,np.int32)
    hc.hc_fit_segments(qcm.ctypes.data,n,nd,guess.ctypes.data,CONSTS.ctypes.data,LAMS.ctypes.data,8,gp.ctypes.data,ss.ctypes.data,gs.ctypes.data,0)
    for k in [35332, 37591, 40458, 66741, 105884]:
        st,po,tol=LC.oracle_fit((nd,qi[k],guess[k]))
        sp4=LC.oracle_spread((nd,qi[k],guess[k],po,4)); sp32=LC.oracle_spread((nd,qi[k],guess[k],po,32))
        d=LC._dist(gp[k][None],po[None])[0]
        print(k,'d/tol',np.round(d/tol,2),'spread4/tol',np.round(sp4/tol,2),'spread32/tol',np.round(sp32/tol,2))

if __name__=="__main__":
    detail() if sys.argv[1:] == ["detail"] else main()
