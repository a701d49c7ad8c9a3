#!/bin/bash
# Decode attention at 32 / 64 lock-step prompts (P = 460): kernel trace + FETCH_SIZE pass.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/attn; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/bench_attn.py 20 --many > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc -o run --output-format csv -- python3 $R/scripts/bench_attn.py 5 --many > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
cd $R
cat $O/trace.log | grep '^{'
python3 - <<'PY'
import csv, glob, collections
R='gpurun_out/attn'
f=glob.glob(R+'/trace/**/*kernel_trace.csv', recursive=True)[0]
g=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'attn' in r['Kernel_Name']:
        g[(r['Kernel_Name'][:40], r['Grid_Size_Z'])].append(int(r['End_Timestamp'])-int(r['Start_Timestamp']))
for k,v in sorted(g.items()): print(k, len(v), round(sum(v)/len(v)/1e3,2),'us')
fs=glob.glob(R+'/pmc/**/*counter_collection.csv', recursive=True)
h=collections.defaultdict(list)
for f in fs:
    for r in csv.DictReader(open(f)):
        if 'attn' in r.get('Kernel_Name',''):
            h[(r['Kernel_Name'][:40], r['Grid_Size'])].append(float(r['Counter_Value']))
for k,v in sorted(h.items()): print('FETCH_SIZE KiB', k, len(v), round(sum(v)/len(v)), '-> x2 MB', round(2*sum(v)/len(v)*1024/1e6,1))
PY
