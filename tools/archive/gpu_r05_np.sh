#!/bin/bash
# Round 5: finish_kernel's polish block count (F2 line, two runs each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
B="--no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0 --tol-run 0"
for np in 1024 512 256 1024 512 256; do
  PHGPU_FIN_NP=$np timeout -k 10 200 python -u bench.py $B > $O/f2_np$np.json 2> $O/f2_np$np.err || { echo "bench failed"; tail -20 $O/f2_np$np.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f2_np$np.json'));print('np $np', d['ms_per_step'], d['roofline']['kernels'])"
done
