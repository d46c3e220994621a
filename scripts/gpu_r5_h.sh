# PMC baseline for the exchange-traffic ratio: lenet_mw (the same batch reductions + update, no
# exchange), same counter groups as gpu_r5_g.sh.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/g_pmc
P1="TCP_TCC_UC_READ_REQ_sum TCP_TCC_UC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
P2="TCC_EA0_RD_UNCACHED_32B_sum TCC_EA0_WR_UNCACHED_32B_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
export MLT_LENET_PREP=0
i=0
for grp in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/g_pmc/base_p$i -o run -- \
    python3 -u bench.py --steps 200 --warmup 20 --no-fp32-companion > gpurun_out/g_pmc/base_p$i.log 2>&1 || exit 1
done
python3 scripts/pmc_summary.py gpurun_out/g_pmc/base_p1 gpurun_out/g_pmc/base_p2 --match lenet_mw --jsonl gpurun_out/g_pmc/base.jsonl > gpurun_out/g_pmc/base.txt
