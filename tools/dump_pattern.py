"""Write a workload's sparsity pattern in the test harnesses' stdin format
("n m nnz", row_ptr, col_idx) followed by "seed fixed_frac inactive_frac
delta".   python tools/dump_pattern.py uc|farmer1000|sslp seed ffix finact delta"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
from mpisppy_amd import batch  # noqa: E402

kind = sys.argv[1]
if kind == "uc":
    from mpisppy_amd.examples import uc
    d = uc.batch_creator(["Scenario1", "Scenario2"])
elif kind.startswith("farmer"):
    from mpisppy_amd.examples import farmer
    c = int(kind[len("farmer"):])
    d = batch.from_models(["scen0", "scen1"], [farmer.scenario_creator(nm, crops_multiplier=c)
                                               for nm in ["scen0", "scen1"]])
else:
    from mpisppy_amd.examples import sslp
    names = sslp.scenario_names(5)[:2]
    d = batch.from_models(names, [sslp.scenario_creator(nm, data_dir="data/sslp_15_45_5/scenariodata")
                                  for nm in names])
n = d.l.shape[0]
out = sys.stdout
out.write(f"{n} {d.m} {len(d.col_idx)}\n")
out.write(" ".join(map(str, d.row_ptr)) + "\n")
out.write(" ".join(map(str, d.col_idx)) + "\n")
out.write(" ".join(sys.argv[2:6]) + "\n")
