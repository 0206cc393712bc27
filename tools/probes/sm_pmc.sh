# PMC passes (own runs, kernel trace only) of the two small-batch sgemv forms on one shape: HBM bytes fetched and
# L2 hit/miss, to see whether the matrix-core form's 64-byte row runs per load instruction re-fetch lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sm_pmc; mkdir -p $O
for form in 5 17; do
  for pass in "FETCH_SIZE TCC_HIT_sum" "TCC_MISS_sum TCC_REQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    tag=mm${form}_$(echo $pass | cut -c1-8)
    K8S_SGEMV_MFMA_MIN_M=$form timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $O/$tag -o run -- python3 tools/probes/sm_pmc.py > $O/$tag.log 2>&1
    rc=$?; echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.log; exit $rc; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/sm_pmc/*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "sgemv" in r["Kernel_Name"] or "smfma" in r["Kernel_Name"]:
            agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f.split("/")[2], k, c, f"{sum(v) / len(v):.4g}")
PY
