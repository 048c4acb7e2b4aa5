#!/bin/bash
# GPU-box run of the parity suite (-m gpu), verbose log under gpurun_out/.  Extra pytest args: $@.
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 \
    --timeout-method thread --durations=25 "$@" > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -40 gpurun_out/tests.log
exit $rc
