#!/bin/bash
# rocprofv3 kernel-trace + stats of a command, CSV into gpurun_out/<name>/ (run from the repo root).
# usage: tools/prof.sh NAME python3 tools/cg_only.py arm 50000 20
name=$1; shift
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
exec_args=("$@")
case "${exec_args[1]}" in /*) ;; *) exec_args[1]="$root/${exec_args[1]}";; esac
rocprofv3 --kernel-trace --stats --output-format csv -d "$root/gpurun_out/$name" -o run -- "${exec_args[@]}"
