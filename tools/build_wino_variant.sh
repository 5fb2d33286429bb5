# Build a variant of the library with extra defines on one source, for A/B
# runs through tools/wino_pmc.py --lib:
#   bash tools/build_wino_variant.sh NAME SRC "-DFOO=1 -DBAR=2"
# -> tools/hip/v_NAME.so (git-ignored; travels to the GPU box)
set -e
NAME=$1; SRC=$2; DEFS=$3
cd "$(dirname "$0")/../scaled-mmd-gan_amd/csrc"
make -s
OBJ=/tmp/v_${NAME}_$(basename $SRC .hip).o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function \
  -munsafe-fp-atomics -I../../include $DEFS -c $SRC -o $OBJ
OBJS=$(ls build/*.o | grep -v "build/$(basename $SRC .hip).o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/hip/v_${NAME}.so $OBJS $OBJ
echo built tools/hip/v_${NAME}.so
