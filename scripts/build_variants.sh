#!/bin/bash
# Build A/B variants of libggml-mi355x.so in-tree (lib_<name>/, objects in build_<name>/):
#   build_variants.sh name1="-DFOO=0" name2="-DBAR=0 -DFOO=0" ...
# Every variant is an MX_AB_VARIANTS=1 build: the experiment-only code (timing variants,
# debug masks, the balanced QKV layout) the product library leaves out.
cd "$(dirname "$0")/../llama-mi50.cpp_amd"
for spec in "$@"; do
  n=${spec%%=*}; x=${spec#*=}
  # seed with the default objects; rebuild the ones that see the GEMV switches (REBUILD)
  mkdir -p build_$n; cp build/*.o build_$n/ 2>/dev/null
  for f in ${REBUILD:-exec ops_gemv ops_mm ops_qkv ops_mmq4}; do rm -f build_$n/$f.o; done
  make -s -j8 OBJ=build_$n OUT=lib_$n EXTRA="-DMX_AB_VARIANTS=1 $x" > /tmp/build_$n.log 2>&1 || { echo "variant $n failed"; tail -20 /tmp/build_$n.log; exit 1; }
  echo "built lib_$n ($x)"
done
