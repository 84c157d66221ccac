#!/bin/bash
# full -m gpu suite at HEAD
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/r6
TTMO=2400 bash scripts/r6.sh "tests"
