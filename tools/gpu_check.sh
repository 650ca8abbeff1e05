#!/bin/bash
# On the GPU box (gpurun): GPU tests -> smoke -> bench, each step under its own time limit,
# stopping at the first failing step.  Usage: tools/gpu_check.sh [bench args...]
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 700 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
