#!/bin/bash
# round-4 HEAD check after the MX-FP8 group knob: full GPU suite, smoke
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA > gpurun_out/r04f5_gtests.log 2>&1; rc=$?; echo "gtests rc=$rc"; tail -1 gpurun_out/r04f5_gtests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r04f5_gtests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f5_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r04f5_smoke.log

exit $rc
