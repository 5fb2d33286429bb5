# Standalone builds of csrc/smmd_conv1x1.hip for tools/c1_probe.py A/B runs
# (tools/hip/c1_*.so, git-ignored): the shipped source (c1_base), its slicing
# knobs (C1_TARGET, C1_MINCH_GEMM, C1_MINCH_WGRAD), and two diagnostic builds
# made by text substitution in /tmp (MFMAs replaced by one FMA; output stores
# skipped) that split a launch's time between memory and MFMA work.
#   bash tools/build_c1_variants.sh ["NAME:-DDEF=1 -DDEF2=2" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/scaled-mmd-gan_amd/csrc/smmd_conv1x1.hip
O=$R/tools/hip
T=$(mktemp -d)
b() { /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -shared -I$R/include \
      -I$R/scaled-mmd-gan_amd/csrc $2 $1 -o $O/c1_$3.so; }
python3 - "$S" "$T" <<'PY'
import sys
src = open(sys.argv[1]).read()
t = sys.argv[2]
nm = src.replace('acc = __builtin_amdgcn_mfma_f32_32x32x2f32(', 'acc = C1_NOMFMA(')
nm = nm.replace('typedef float f32x16 __attribute__((ext_vector_type(16)));',
                'typedef float f32x16 __attribute__((ext_vector_type(16)));\n'
                '#define C1_NOMFMA(a, b, c, x, y, z) ([&] { f32x16 t_ = (c); '
                't_[0] = fmaf((a), (b), t_[0]); return t_; }())')
open(t + '/nomfma.hip', 'w').write(nm)
ns = src.replace('yc[(int64_t)(mr + (r & 3) + 8 * (r >> 2)) * P] = acc[r];',
                 'if (acc[r] == -1.2345e-37f) yc[(int64_t)(mr + (r & 3) + 8 * (r >> 2)) * P] = acc[r];')
assert ns != src
open(t + '/nostore.hip', 'w').write(ns)
PY
b $S "" base
b $T/nomfma.hip "" nomfma
b $T/nostore.hip "" nostore
for v in "$@"; do b $S "${v#*:}" "${v%%:*}"; done
rm -rf "$T"
ls $O/c1_*.so
