# instruction-cache counters of the layered decoder (dev probe): one pass per counter pair
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03j}
mkdir -p $OUT
cd /tmp
i=0
for ctr in "SQC_ICACHE_REQ SQC_ICACHE_MISSES" "SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/tools/probe.py layered 4096 > $OUT/pmc$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $OUT/pmc$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob, os, collections
out = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("TAG", "r03j")
for f in sorted(glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "ldpc_dec_kernel_l" not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    disp = {k: v / max(1, len({})) for k, v in agg.items()}
    print(os.path.relpath(f, out), {k: f"{v:.4g}" for k, v in agg.items()})
PY
