#!/bin/bash
# GPU gate on the box: the -m gpu suite, then (unless the suite crashed or hung) the default bench.
# pytest exit 1 = some tests failed (the GPU is fine: the bench still runs); any other non-zero
# status (fault, abort, timeout) ends the script.  Usage: tools/gpu_gate.sh TAG [bench args...]
tag=${1:-gate}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
brc=$?
tail -c 600 gpurun_out/${tag}_bench.json
[ $brc -ne 0 ] && exit $brc
exit $rc
