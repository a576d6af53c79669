#!/bin/bash
# chol_df timelines (M3S_DF_STAMPS diagnostic build, plain launch) for cfg3's and cfg4's core sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05y
mkdir -p $O
for n in 192 896; do
timeout -k 10 120 tools/bin/ubench_chol_df $n 5 > $O/df_$n.log 2>&1 || { echo "ubench rc=$?"; tail -5 $O/df_$n.log; exit 1; }
cat $O/df_$n.log | head -40
done
