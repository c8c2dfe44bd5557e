#!/bin/bash
# Freeze the working tree (sources, built libraries, tests, tools) into ab/run/ so a queued GPU call runs one
# consistent build even if the tree keeps changing while the call waits for a box: GPU steps then run as
# 'cd ab/run && ...' (ab/ is git-ignored).  usage: bash tools/snap.sh
set -e
cd "$(dirname "$0")/.."
rm -rf ab/run
mkdir -p ab/run
tar --exclude=./ab --exclude=./gpurun_out --exclude=./.git --exclude='*.log' --exclude=./vit-cnn_amd/csrc/build -cf - . | tar -xf - -C ab/run
echo "snapshot ab/run: $(du -sh ab/run | cut -f1)"
