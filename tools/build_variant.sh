#!/bin/bash
# Build an A/B variant of libgpk with extra defines: tools/build_variant.sh OUT.so -DFOO=1 ...
out=$1; shift
S=gaussianprocessfundamentals_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value -Iinclude -I$S "$@" \
  $S/gpk_assemble.hip $S/gpk_diag.hip $S/gpk_potrf.hip $S/gpk_approx.hip $S/gpk_eig.hip $S/gpk_flat.hip $S/gpk_abi.hip -o "$out"
