set -o pipefail
T=${1:-r}
bash tools/r06/ab_env.sh $T 2 "" keep="M3S_GN_PCG=1" nokeep="M3S_POOL_KEEP_MB=0" pcg3="M3S_GN_PCG=2" pcg3_nokeep="M3S_GN_PCG=2 M3S_POOL_KEEP_MB=0" direct="M3S_GN_PCG=0"
