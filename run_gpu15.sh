#!/bin/bash
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu15.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu15.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/phaseprof.py jobs > gpurun_out/phasejobs15.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench15.log 2>&1
