#!/bin/bash
# round 3: DenseNet conv / wgrad staging with batched loads -- parity tests, smoke loss, densenet bench leg
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ao}
timeout -k 10 400 python -u -m pytest tests/test_densenet_gpu.py tests/test_trajectories_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_${T}.log 2>&1 && tail -3 gpurun_out/tests_${T}.log && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 && cat gpurun_out/smoke_${T}.log && \
timeout -k 10 300 python -u bench.py --workload densenet --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/bench_dn_${T}.json 2> gpurun_out/bench_dn_${T}.err && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_dn_${T}.json') if x.startswith('{')][-1]; d=json.loads(l); v=d.get('densenet', d); print('densenet', v.get('value'), v.get('ms_per_step'), (v.get('roofline') or {}).get('frac'))"
