#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
bash scripts/gpurun/r5_i.sh || exit 1
bash scripts/gpurun/r5_j.sh || exit 1
