#!/bin/bash
# attention parity tests + the many-prompt microbench (kernel trace) + the 64-prompt AR line
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/attnq; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_attn_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/scripts/bench_attn.py 20 --many $ATTN_P > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cd $R; grep '^{' $O/trace.log | cut -c1-200
python3 - <<'PY'
import csv, glob, collections
f=glob.glob('gpurun_out/attnq/trace/**/*kernel_trace.csv', recursive=True)[0]
g=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'attn' in r['Kernel_Name']:
        g[(r['Kernel_Name'][:40], r['Grid_Size_X'], r['Grid_Size_Z'])].append(int(r['End_Timestamp'])-int(r['Start_Timestamp']))
for k,v in sorted(g.items()): print(k, len(v), round(sum(v)/len(v)/1e3,2),'us')
PY
[ -z "$NO_AR" ] && bash scripts/gpu_quick2.sh || true
