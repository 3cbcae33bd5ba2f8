#!/bin/bash
# rocprofv3 passes over a short bench run: kernel-trace stats, then one PMC pass per counter
# group (FETCH_SIZE and WRITE_SIZE cannot share a pass; MI355X_MICROARCH.md "rocprofv3 PMC slots").
# Usage: tools/profile.sh <tag> [bench args...]   -> gpurun_out/prof_<tag>/...
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --cpu-budget 0 "$@" > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py --cpu-budget 0 "$@" > $out/fetch.log 2>&1 || { tail -20 $out/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py --cpu-budget 0 "$@" > $out/write.log 2>&1 || { tail -20 $out/write.log; exit 1; }
find $out -name '*.csv' | sort
