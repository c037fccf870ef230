"""Fit the FFD candidate-loop cost model on a per-batch timeline (tools/pipe_stats.py TIMELINE=...):
cycles = a*checks + b*hits + c*todo + d, plus stage concurrency.  Usage: python tools/tl_fit.py tl.csv ..."""
import sys

import numpy as np
import pandas as pd

for path in sys.argv[1:]:
    d = pd.read_csv(path)
    cand = (d.t_cand - d.t_prescan).to_numpy(float)
    X = np.c_[d.checks, d.hits, d.todo, np.ones(len(d))]
    coef = np.linalg.lstsq(X, cand, rcond=None)[0]
    r2 = 1 - ((X @ coef - cand) ** 2).sum() / ((cand - cand.mean()) ** 2).sum()
    span = (d.t_cand.max() - d.t_ready.min()) / 1e6
    print(f"{path}: span {span:.2f} Mcyc, cand {cand.sum()/1e6:.2f} Mcyc, prescan {(d.t_prescan-d.t_ready).sum()/1e6:.2f} Mcyc,"
          f" checks {d.checks.sum()} hits {d.hits.sum()} todo {d.todo.sum()} | per check {coef[0]:.0f} per hit {coef[1]:.0f}"
          f" per todo {coef[2]:.0f} per batch {coef[3]:.0f} (R2 {r2:.3f})")
