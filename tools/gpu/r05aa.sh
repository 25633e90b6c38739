set -o pipefail
# round 5, run aa: where p4<32>'s LDS bank conflicts come from -- SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS of the <32> launches
# under the diagnostic ablations (conv_dbg 4096 | AB << 13: AB 16 no B reads, 4 no epilogue, 2 no GroupNorm transform)
R=r05aa
mkdir -p gpurun_out/$R
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 135168 36864 20480; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/$R/p_$v -o run -- python3 tools/census.py --reps 1 --n 256 --lib ab_libs/libitsd_hip_diag.so --set conv_dbg=$v > gpurun_out/$R/p_$v.log 2>&1 || { echo pmc_fail $v; tail -3 gpurun_out/$R/p_$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for v in (0, 135168, 36864, 20480):
    f = glob.glob(f"gpurun_out/r05aa/p_{v}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for fn in f:
        for r in csv.DictReader(open(fn)):
            if "conv3x3_gn_p4_kernel<32" in r["Kernel_Name"]:
                acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = collections.defaultdict(float)
    for d in acc.values():
        for k, x in d.items(): tot[k] += x
    nd = max(len(acc), 1)
    print(v, "dispatches", len(acc), {k: "%.3g" % (x / nd) for k, x in tot.items()})
PY
