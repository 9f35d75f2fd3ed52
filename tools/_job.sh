set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x --timeout 300 --timeout-method thread -q tests -m gpu -k "byte or bytes or band or tiled or config" > gpurun_out/pytest_sub.log 2>&1 || { tail -40 gpurun_out/pytest_sub.log; exit 3; }
tail -2 gpurun_out/pytest_sub.log
rm -f gpurun_out/ab4.log
for W in "--workload byte16k --steps 600" "--steps 20" "--workload strong262k --steps 20" "--workload bit64k --steps 100"; do
  L=tools/variants/libr05a.so,lib
  case "$W" in *byte16k*) L=tools/variants/libr05a.so,tools/variants/libbpair4.so,tools/variants/libbpair6.so,lib;; esac
  timeout -k 10 600 python tools/ab.py --reps 3 --libs $L --bench "$W" >> gpurun_out/ab4.log 2>&1 || { tail -20 gpurun_out/ab4.log; exit 4; }
done
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('gpurun_out/ab4.log'):
    if l.startswith('{'):
        d=json.loads(l); r[(d['bench'],d['lib'])].append((d['value'], d['alive_final']))
for k,v in r.items(): print(k, [round(x[0]/1000,1) for x in v], set(x[1] for x in v))
"
