"""Round 6 analysis: how many of C2's complete trees a single-pass fold with candidate binades from
each row block's first-tile sum would cover (CPU, the oracle's predictions; prints the offsets
between the plan's binade and the estimate's)."""
import sys, numpy as np, time
sys.path[:0]=['symbolicregression.jl_amd','oracle','.']
from sr_amd import Options, flatten_trees, gen_random_population
from oracle import Oracle
import bench
n=1<<20
X,y=bench.c2_data(n,0)
opts=Options(**bench.C2_OPS)
trees=gen_random_population(10000, opts, 5, max_size=30, seed=1)
tb=flatten_trees(trees,np.float32)
orc=Oracle.from_options(opts)
L, C = orc.eval_loss_batch(tb, X, y, accum="f64", n_threads=8)
idx=np.nonzero(C & np.isfinite(L))[0][::6]
rb=4096; tile=1024; dd=2.0**-8
def q(x): return np.floor(np.log2(np.maximum(x,1e-300)))
offs=[]; fails={1:0,2:0,3:0,4:0}; fails_est2={1:0,2:0,3:0}; nt=0
for k in idx:
    p, ok = orc.eval_tree_array(tb, int(k), X)
    d=(p-y).astype(np.float32); l=(d*d).astype(np.float64)
    segs=l.reshape(-1,rb).sum(1)
    t0s=l.reshape(-1,tile).sum(1)[::rb//tile]
    Sb=np.concatenate([[0.0],np.cumsum(segs)])
    qa=q(Sb[:-1]*(1-dd)); qb=q(Sb[1:]*(1+dd))
    steps=(qa==qb); steps[0]=False
    j=np.arange(len(segs))
    est=j*(rb//tile)*t0s
    o=(qa-q(est))[steps]
    offs.append(o)
    nt+=1
    for K in fails:  # candidates q_base-1 .. q_base+K-2
        if np.any((o< -1)|(o> K-2)): fails[K]+=1
print("trees",nt,"fails by K (cands -1..K-2):",fails)
o=np.concatenate(offs); u,c=np.unique(o,return_counts=True); print(dict(zip(u.astype(int).tolist(),c.tolist())))
