cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/r05_e3 -o run -- python3 tools/bench_split.py --set main --iters 5 > gpurun_out/r05_e3.log 2>&1 || { tail -5 gpurun_out/r05_e3.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/r05_e3/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])[:10]:
    w = max(v["SQ_WAVES"], 1)
    print("%-70s waves %8d wcyc/w %8.0f ic_miss/w %6.1f ic_hit/w %8.1f ifetch/w %8.1f winst%% %5.1f" % (
        k, w, v["SQ_WAVE_CYCLES"] / w, v["SQC_ICACHE_MISSES"] / w, v["SQC_ICACHE_HITS"] / w, v["SQ_IFETCH"] / w,
        100 * v["SQ_WAIT_INST_ANY"] / max(v["SQ_WAVE_CYCLES"], 1)))
PY
rm -rf gpurun_out/r05_e3
