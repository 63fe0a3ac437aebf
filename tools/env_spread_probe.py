"""Spread of one env's oracle result under rounding-scale perturbations (CPU; the full-state rule's
envelope, tests/test_gpu_fullstate.py). Rebuilds the 65 536-env check of
tests/test_gpu_fullsize.py::test_full_state_headline_sizes, takes sample column 99 (env 6192, the
env round 4's GPU run r4g left unexplained with a 29.5 N feet-force deviation) and prints its f32 /
f64 oracle force rows and the distribution of the first force row over thousands of perturbed runs
(profiles/r4g/env99_oracle_spread.txt). Run from the repo root: python tools/env_spread_probe.py
"""
import sys, numpy as np
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
from fullstate import random_states, task_cfg, row_groups, perturb_physics
from oracle.pyoracle import OracleSim
from test_gpu_fullsize import _sample
n=65536; task='v2'; seed=29
st = random_states(task, OracleSim(n, task_cfg(task), seed=seed), n, seed=300+n)
a = np.random.default_rng(n).normal(size=(n, 6)).astype(np.float32)
ids=_sample(n); e=ids[99]; print("env id", e)
s1=np.ascontiguousarray(st[:, [e]]); a1=np.ascontiguousarray(a[[e]])
fr=row_groups(task)["force"]
def run(stt, double=False):
    o=OracleSim(1, task_cfg(task), seed=seed, double=double); o.set_state(stt); o.step(a1); return o.get_state()[:,0]
base=run(s1); d=run(s1,True)
print("force rows f32", base[fr][:4], "f64", d[fr][:4])
rng=np.random.default_rng(0)
for sc,(rel,ab) in (("1e-6",(1e-6,1e-7)),("1e-5",(1e-5,1e-6)),("1e-4",(1e-4,1e-5))):
    vals=[]
    for k in range(200):
        vals.append(run(perturb_physics(s1,rng,rel,ab))[fr][0])
    vals=np.array(vals); print(sc, "force0 min/max", vals.min(), vals.max(), "frac far(>5N)", np.mean(np.abs(vals-base[fr][0])>5))
vals=[]
for k in range(3000):
    sc = 1e-6 if k < 1500 else 1e-5
    vals.append(run(perturb_physics(s1,rng,sc,sc/10))[fr][:4])
vals=np.array(vals)
print("force0 percentiles", np.percentile(vals[:,0],[0,0.1,1,5,50,95,99,99.9,100]))
print("force1 percentiles", np.percentile(vals[:,1],[0,0.1,1,5,50,95,99,99.9,100]))
names=row_groups(task)
print({k: v[:6] for k,v in names.items()})
