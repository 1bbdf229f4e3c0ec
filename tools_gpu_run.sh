#!/bin/bash
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 5 300 python scripts/ab_variant.py bf 900000 16 10 > gpurun_out/ab.log 2>&1; echo rc=$?; tail -3 gpurun_out/ab.log
