#!/bin/bash
set -e
mkdir -p gpurun_out
MJX355_STAMP_MINROWS=61 timeout -k 10 200 python scripts/stage_profile.py > gpurun_out/s2_stages_heavy2.txt 2>&1
