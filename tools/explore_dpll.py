import sys, time
sys.path.insert(0,'sat-mpi-stana-andrei_amd'); sys.path.insert(0,'oracle')
import numpy as np
from satmi import cnf
from satmi.dpll import dpll_batch
for (n,k,alpha,B) in [(50,3,4.26,4096),(100,3,4.26,4096),(150,3,4.26,512),(200,5,21.0,16),(250,3,4.26,64)]:
    m=int(round(alpha*n)); batch=cnf.uniform_ksat(B,n,m,k,seed=1)
    t=time.time(); r=dpll_batch(batch,mode='sound',max_solutions=1,time_limit=30.0); dt=time.time()-t
    c=r.counters
    print(f"n={n} k={k} B={B}: {dt:.3f}s  {B/dt:.1f} inst/s  sat={int((c[:,5]>0).sum())} nodes/inst={c[:,0].mean():.0f} max={c[:,0].max()} props/inst={c[:,2].mean():.0f} timeouts={(r.status==3).sum()}", flush=True)
