#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AUT_ROUNDS=3000 timeout -k 10 240 python -u profiles/race_autopsy.py > gpurun_out/r05_autopsy.jsonl 2> gpurun_out/r05_autopsy.log || exit 1
bash profiles/r05_race_ab3.sh nofast noloose
