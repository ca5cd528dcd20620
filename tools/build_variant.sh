#!/bin/bash
# Build an A/B variant of libgpk with extra defines: tools/build_variant.sh OUT.so -DFOO=1 ...
# (per-source objects in parallel, under gaussianprocessfundamentals_amd/_obj_<flags>/; see _build.py)
out=$1; shift
exec python3 gaussianprocessfundamentals_amd/_build.py -o "$out" "$@"
