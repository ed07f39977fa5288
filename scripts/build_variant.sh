#!/bin/bash
# Build a variant of libwhisper_mi355x.so for on-GPU A/B runs (scripts/session.sh ab=WMI_LIB=...,
# scripts/lib_equal.py):
#   bash scripts/build_variant.sh NAME "PERSIST_FLAGS" ["EXTRA"]
# -> whisper.rs_amd/ab/NAME/libwhisper_mi355x.so (select it with WMI_LIB)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1
make -s -C $R/whisper.rs_amd/csrc -j8 BUILD=$R/whisper.rs_amd/ab/$N/build OUT=$R/whisper.rs_amd/ab/$N/libwhisper_mi355x.so \
  PERSIST_FLAGS="$2" EXTRA="$3"
echo "built $N"
