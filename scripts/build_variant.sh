# Builds a variant of libdeltareplay.so with extra compile definitions into var_libs/<name>/
# (for scripts/gpu_kvariants.sh, scripts/gpu_snapvar.sh): scripts/build_variant.sh <name> "-DX=1 -DY=2"
set -e
name=$1; defs=$2
mkdir -p var_libs/$name
make -j8 -s OBJDIR=build/var_$name LIB=var_libs/$name/libdeltareplay.so \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable $defs" \
  var_libs/$name/libdeltareplay.so
