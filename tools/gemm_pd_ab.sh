#!/bin/bash
# k-major GEMM register-set depth A/B on single shapes (tools/gemm_one.py, HIP events)
export VITCNN_LIB=${VITCNN_LIB:-$(pwd)/vit-cnn_amd/vitcnn_amd/libvitcnn_probe.so}  # measurement knobs: the probe library
for shape in "0 1 5184 144 144" "0 1 5184 144 256" "0 0 5184 144 256" "0 1 3136 256 512" "0 1 51840 41 72" "1 0 144 144 5184" "0 1 1600 72 144" "0 1 3136 256 1296" "0 0 51840 72 41"; do
  for pd in 1 2; do
    echo "PD=$pd $(VITCNN_GEMM_PD=$pd timeout -k 5 60 python tools/gemm_one.py $shape 4 300)"
  done
done
