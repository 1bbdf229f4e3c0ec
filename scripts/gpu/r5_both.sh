#!/bin/bash
set -o pipefail
bash scripts/gpu/r5_dist.sh && bash scripts/gpu/r5_base.sh
