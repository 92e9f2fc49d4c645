#!/bin/bash
# PMC traffic (FETCH_SIZE, WRITE_SIZE passes) and MFMA busy (one pass) of several calls of one config, each pass its
# own rocprofv3 run under a hard time limit; stops at the first failure.
# usage: tools/pmc_calls.sh <config> '<label1>' ['<label2>' ...]   (labels: full 'prog[i]:function')
set -e
cfg=$1; shift
for label in "$@"; do
  bash tools/pmc_traffic.sh "$cfg" "$label"
  bash tools/pmc_mfma.sh "$cfg" "${label%%:*}"
done
