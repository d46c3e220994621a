# A/B of the GEMM grouped-raster width (MLT_GEMM_GROUP_M) on the transformer benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && : > gpurun_out/ab_groupm.log
for g in 8 4 16; do
  MLT_GEMM_GROUP_M=$g timeout -k 10 150 python3 -u bench.py --model large --steps 8 --warmup 3 > gpurun_out/gm_large_$g.log 2>&1 || exit $?
  echo "large g=$g $(grep -o '"value": [0-9.]*' gpurun_out/gm_large_$g.log)" >> gpurun_out/ab_groupm.log
  MLT_GEMM_GROUP_M=$g timeout -k 10 150 python3 -u bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/gm_base_$g.log 2>&1 || exit $?
  echo "bert-base g=$g $(grep -o '"value": [0-9.]*' gpurun_out/gm_base_$g.log)" >> gpurun_out/ab_groupm.log
done
