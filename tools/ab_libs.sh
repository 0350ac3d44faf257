#!/bin/bash
# A/B two builds of libvonoma.so on the MRF kernels: tools/ab_libs.sh BASE_SO NEW_SO ab_pair2-args...
base=$1; new=$2; shift 2
for lib in "$base" "$new"; do
  echo "### $lib"
  VO_LIB_PATH=$lib timeout -k 10 300 python -u tools/ab_pair2.py "$@" || exit 1
done
