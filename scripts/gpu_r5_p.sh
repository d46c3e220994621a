# kernel-trace gaps at hipGraph boundaries: bench --steps 40 --warmup 5 (5 steps per graph) under
# rocprofv3 --kernel-trace; also the host time of one replay call (no sync) per graph length
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 -u bench.py --steps 40 --warmup 5 \
  --steps-per-graph 5 --no-fp32-companion > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r5p/tr/**/run_kernel_trace.csv", recursive=True) or glob.glob("gpurun_out/r5p/tr/run_kernel_trace.csv")
rows = [r for r in csv.DictReader(open(f[0])) if "lenet_m" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-80:]  # the timed 40 steps (2 kernels each)
gaps = []
for a, b in zip(rows, rows[1:]):
    gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"]), a["Kernel_Name"][:22], b["Kernel_Name"][:22]))
ks_kw = [g for g, a, b in gaps if "lenet_ms" in a]
kw_ks = [g for g, a, b in gaps if "lenet_ms" in b]
print("KS->KW gaps ns:", sorted(ks_kw)[:3], "...", sorted(ks_kw)[-3:])
print("KW->KS gaps ns (sorted):", sorted(kw_ks))
dur = {}
for r in rows:
    dur.setdefault(r["Kernel_Name"][:22], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in dur.items():
    print(k, "avg ns", sum(v) / len(v))
PY
rm -rf $O/tr
