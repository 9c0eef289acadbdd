#!/bin/bash
mkdir -p gpurun_out/$1
timeout -k 10 200 python -u tools/stamps.py 256 > gpurun_out/$1/stamps.log 2>&1; rc=$?; cat gpurun_out/$1/stamps.log; exit $rc
