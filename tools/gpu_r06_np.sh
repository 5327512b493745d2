#!/bin/bash
# Round 6: finish_kernel's polish block count (PHGPU_FIN_NP) on the F2 line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for rep in 1 2; do
  for np in 256 512 1024 2048; do
    PHGPU_FIN_NP=$np timeout -k 10 200 python3 bench.py --no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0 > $O/np$np.json 2> $O/np$np.err || { echo "np $np failed"; tail -5 $O/np$np.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/np$np.json'));print('NP=$np', d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'])"
  done
done
echo ALLDONE
