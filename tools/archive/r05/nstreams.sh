#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u tools/archive/r05/nstreams.py 2>&1 | grep -v amdgpu.ids
