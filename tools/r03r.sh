# Config-4 level anatomy at DT = 2: kernel trace of 2 fixed-damping trials (tools/dist_model.py) -> per-launch
# durations of k_chol_step by level parity; plus the trailing-free timing variant (CHOL_VARIANT=3).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=$PWD/pan-tilt-zoom-slam_amd
rm -rf gpurun_out/r03r_trace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03r_trace -o run --output-format csv -- python tools/dist_model.py --config config4 --worlds 1 --trials 2 > gpurun_out/r03r_trace.jsonl 2> gpurun_out/r03r_trace.err || { echo TRFAIL; tail gpurun_out/r03r_trace.err; exit 1; }
find gpurun_out/r03r_trace -name "*kernel_trace.csv" | head -1 > gpurun_out/r03r_trace_path.txt
PTZBA_LIB=$P/libptzba_cv3.so timeout -k 10 300 python tools/dist_model.py --config config4 --worlds 1 --trials 6 > gpurun_out/r03r_cv3.jsonl 2> gpurun_out/r03r_cv3.err || { echo FAIL; tail gpurun_out/r03r_cv3.err; exit 1; }
cut -c1-220 gpurun_out/r03r_cv3.jsonl
python - <<'PY'
import csv
p = open('gpurun_out/r03r_trace_path.txt').read().strip()
rows = list(csv.DictReader(open(p)))
ks = [r for r in rows if 'k_chol_step' in r['Kernel_Name']]
d = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in ks]
g = [int(r.get('Grid_Size_X', r.get('Grid_Size', 0)) or 0) for r in ks]
print(len(ks), 'k_chol_step launches')
last = d[-265:]; lg = g[-265:]
import statistics as st
ev = [x for i, x in enumerate(last) if i % 2 == 0]; od = [x for i, x in enumerate(last) if i % 2 == 1]
print('even levels: mean %.1f us  odd: mean %.1f us' % (st.mean(ev) / 1e3, st.mean(od) / 1e3))
print('first 12 levels (us, grid):', [(round(x / 1e3, 1), y // 256) for x, y in zip(last[:12], lg[:12])])
print('levels 130-141:', [(round(x / 1e3, 1), y // 256) for x, y in zip(last[130:142], lg[130:142])])
PY
