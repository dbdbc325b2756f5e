#!/bin/bash
# Round-6 AP: the reference entry scripts re-measured on the end-of-round code.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rm -f gpurun_out/r6_entry_scripts_final.jsonl
timeout -k 10 600 python scripts/entry_scripts_measure.py gpurun_out/r6_entry_scripts_final.jsonl > gpurun_out/r6ap_entry.log 2>&1 || { tail -40 gpurun_out/r6ap_entry.log; exit 1; }
tail -8 gpurun_out/r6ap_entry.log
