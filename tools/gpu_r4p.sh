#!/bin/bash
# Round 4 combined: AR diagnostics (r4n), c3 chain codegen A/B (r4o), then the validation suite (r4d)
set -u
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1, stopping"; exit $1;; esac; }
bash tools/gpu_r4n.sh; rc=$?; fatal $rc
bash tools/gpu_r4o.sh; rc=$?; fatal $rc
bash tools/gpu_r4d.sh; exit $?
