# PMC of the fused xGMI exchange (lenet_mwx, loopback, no prep blocks): memory request counts vs
# the useful granule bytes, for the lane-contiguous granule layout (in-tree .so, "new") and the
# round-4 flat-offset layout (ab/ .so built with -DMLT_XCH_FLAT, "old"). One pass per counter group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/g_pmc
SO=$(ls ml_trainer_amd/_C*.so)
cp "$SO" /tmp/g_new.so
P1="TCP_TCC_UC_READ_REQ_sum TCP_TCC_UC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
P2="TCC_EA0_RD_UNCACHED_32B_sum TCC_EA0_WR_UNCACHED_32B_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
export MLT_LENET_PREP=0
for v in new old; do
  if [ "$v" = new ]; then cp /tmp/g_new.so "$SO"; else cp ab/_C*.so "$SO"; fi
  i=0
  for grp in "$P1" "$P2"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/g_pmc/${v}_p$i -o run -- \
      python3 -u bench.py --transport xgmi-loopback --steps 200 --warmup 20 --no-fp32-companion > gpurun_out/g_pmc/${v}_p$i.log 2>&1 || { cp /tmp/g_new.so "$SO"; exit 1; }
  done
  python3 scripts/pmc_summary.py gpurun_out/g_pmc/${v}_p1 gpurun_out/g_pmc/${v}_p2 --match lenet_mwx --jsonl gpurun_out/g_pmc/$v.jsonl > gpurun_out/g_pmc/$v.txt
  timeout -k 10 120 python3 -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion > gpurun_out/g_pmc/${v}_lb4.log 2>&1 || { cp /tmp/g_new.so "$SO"; exit 1; }
done
cp /tmp/g_new.so "$SO"
