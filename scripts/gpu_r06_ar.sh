#!/bin/bash
# r06 session ar: the whole GPU suite + smoke (dgfwd, DenseNet bnfuse)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/ar_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/ar_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ar_smoke.log 2>&1
