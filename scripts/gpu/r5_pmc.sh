#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
for cfg in "32 10000000" "32 900000" "16 900000"; do
  set -- $cfg
  echo "=== pmc K=$1 N=$2"
  bash tools/profile.sh pmc $1 $2 | grep -v "^summary" || exit 1
done
