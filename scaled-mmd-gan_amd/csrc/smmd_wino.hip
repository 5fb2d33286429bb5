// smmd_wino.hip -- 3x3 stride-1 SAME convolutions as Winograd F(2x2, 3x3) on
// the f32 MFMA (gfx950), fused: input transform, the 16 transform-point GEMMs
// and the output transform in ONE launch, nothing but x, the transformed
// filter and y touching HBM.
//
// The critic's and generator's 3x3 convs (gan/core/resnet/block.py:38-50,
// snops.py:60-80 conv2d with padding SAME; C, K in {64 .. 512}, H = W in
// {8 .. 64}) are the largest single class of step time.  MIOpen runs them as
// F(2,3) Winograd on the VALU (55 TF/s executed, 0.35 of the f32 peak); the
// multiply stage here is `v_mfma_f32_32x32x2_f32` (exact f32 fma chains).
//
//   y[n][k][2ty+a][2tx+b] = bias[k] + (A^T M A)[a][b],
//   M_p[k][t] = sum_c U_p[k][c] V_p[c][t]          (16 points p = 4 i + j)
//   V = B^T d B  (d: the 4x4 input patch at (2ty-1, 2tx-1), zero outside)
//   U = G g G^T  (g: the 3x3 filter [k][c]; the backward-data conv uses the
//                 flipped, transposed filter, mode 1 of the filter transform)
//
// Block: 64 tiles (lanes of the transform waves) x 64 output channels, 4
// waves; wave w computes the 32 x 32 (k, tile) quadrant (kh = w >> 1, th =
// w & 1) for all 16 points: 16 f32x16 accumulators (256 AGPRs), so for one
// (k, tile) every point lives in the same lane and register and the output
// transform runs in registers.  Input channels go 8 per chunk through a
// double-buffered LDS stage (V 32 KB + U 32 KB per buffer): chunk c+1's
// global loads are issued before chunk c's 64 MFMAs per wave; its transform
// and LDS stores are cut into 32 slices issued one after each of the second
// half's MFMAs (in the matrix core's shadow), one barrier per chunk.
// Measured and not kept: a 16x16x4 form with 32 output channels per block,
// 128 accumulator registers and two workgroups per CU (129 / 110 / 101 / 118
// us vs 132 / 112 / 97 / 102 us on the four SNResNet-64 layers).
#include "smmd_common.hpp"
#include "smmd_ldsdma.hpp"

namespace smmd {

namespace {

constexpr int WN_T = 256;                 // threads per block
constexpr int WN_TB = 64;                 // tiles per block
constexpr int WN_KB = 64;                 // output channels per block
constexpr int WN_CC = 8;                  // input channels per chunk
constexpr int WN_STAGE = 16 * WN_CC * 64; // floats per V (and per U) stage
// + the block's 64 biases: the epilogue reads them from LDS, so its rows never
// wait on a global load (a load there waits, in order, for every earlier store)
constexpr size_t WN_LDS = 2 * 2 * WN_STAGE * sizeof(float) + WN_KB * sizeof(float) +
                          2 * 2 * 16 * sizeof(float);   // (+ the 8-wave kernel's V padding)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

// neighbour lanes' values, 0 where the source lane is outside the wave
// (bound_ctrl: no preset of the destination)
__device__ __forceinline__ float wn_dpp_left(float v) {    // lane l gets lane l-1's v
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138,
                                                              0xf, 0xf, true));
}

__device__ __forceinline__ float wn_dpp_right(float v) {   // lane l gets lane l+1's v
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x130,
                                                              0xf, 0xf, true));
}

// U = G g G^T for the filters (ko, 4 q .. 4 q + 3), stored in the conv
// kernel's LDS order u[kb][chunk][p][h][k64][c4] (c = 4 h + c4 within the
// chunk of 8): a thread owns one ko and four consecutive ci, so each point's
// four values are one float4 store and consecutive lanes (consecutive ko)
// store consecutive 16 bytes
//
// sig != NULL (smmd_wino3x3_filter_sn): w is the raw weight W of a spectrally
// normalised layer and the filter is W_eff = (W / sigma) * s, formed here with
// the SN refresh's own arithmetic (sn.py:43, snops.py:84; smmd_sn.hip P3, no
// contraction), so U is bit-identical to the transform of a stored W_eff and
// the refresh need not write W_eff at all.
__global__ void wino_filter_kernel(const float *__restrict__ w, int KO, int CI, int mode,
                                   float *__restrict__ u, const float *__restrict__ sig,
                                   const float *__restrict__ sc) {
#pragma clang fp contract(off)
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)KO * (CI >> 2)) return;
    const int ko = (int)(idx % KO), q = (int)(idx / KO);
    const float sigma = sig ? sig[0] : 1.f, scale = sc ? sc[0] : 1.f;
    float r[16][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int ci = 4 * q + e;
        float g[3][3];
        if (mode == 0) {
            const float *s = w + ((int64_t)ko * CI + ci) * 9;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) g[i][j] = s[i * 3 + j];
        } else {        // w is [CI][KO][3][3] of the forward conv; flip both taps
            const float *s = w + ((int64_t)ci * KO + ko) * 9;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) g[i][j] = s[(2 - i) * 3 + (2 - j)];
        }
        if (sig) {
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) g[i][j] = (g[i][j] / sigma) * scale;
        }
        float t[4][3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            t[0][j] = g[0][j];
            t[1][j] = 0.5f * (g[0][j] + g[1][j] + g[2][j]);
            t[2][j] = 0.5f * (g[0][j] - g[1][j] + g[2][j]);
            t[3][j] = g[2][j];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            r[i * 4 + 0][e] = t[i][0];
            r[i * 4 + 1][e] = 0.5f * (t[i][0] + t[i][1] + t[i][2]);
            r[i * 4 + 2][e] = 0.5f * (t[i][0] - t[i][1] + t[i][2]);
            r[i * 4 + 3][e] = t[i][2];
        }
    }
    const int kb = ko >> 6, kl = ko & 63, cc = q >> 1, h = q & 1;
    float4 *u4 = reinterpret_cast<float4 *>(u);
    const int64_t base = ((int64_t)kb * (CI >> 3) + cc) * 16;
#pragma unroll
    for (int p = 0; p < 16; ++p)
        u4[((base + p) * 2 + h) * 64 + kl] = make_float4(r[p][0], r[p][1], r[p][2], r[p][3]);
}

struct WnGeom {
    int N, C, K, H, W, TW, Timg;
    int64_t T, slab;        // slab: floats between split-C partial outputs
    int relu;               // 1: the output is relu(conv + bias) (not on partial slabs);
                            // 2: mask <= 0 ? 0 : conv + bias (threshold_backward's select)
    const float *mask;      // relu 2: of y's shape (smmd_wino3x3_conv_mask)
    // the pair form (smmd_wino3x3_conv2): a second input and filter, the
    // input-channel loop running over both (chunks nch1 .. 2 nch1 - 1 from
    // them), so y = conv(x, U) + conv(x2, U2) in one set of accumulators
    const float *x2, *u2;
    // the 8-wave kernel's 1-D grid: tile blocks, output-channel blocks,
    // input-channel slices (w8_block)
    int TB, KB, S;
};

// The input transform V = B^T d B of one tile's 4 x 4 patch d (rows 2ty-1 ..
// 2ty+2, columns 2tx-1 .. 2tx+2), factored by columns: t = B^T d column by
// column, v = t B row by row.  A lane loads only its two centre columns
// (2tx, 2tx+1); t's outer columns are the neighbouring tiles' centre columns,
// so they come transformed from the neighbour lanes (t[.][0] = the left
// tile's t of its column 2tx-1, t[.][3] = the right tile's t of 2tx+2):
// 8 column ops instead of 16 and no raw neighbour values.  Rows 1 and 2 are
// always inside the image (H even); rows 0 and 3 are zero at its top and
// bottom, columns 0 and 3 at its left and right edges.  The arithmetic is
// the column-then-row form, term for term.

// B^T of one column of the patch
__device__ __forceinline__ void wn_bt(float a0, float a1, float a2, float a3, float (&t)[4]) {
    t[0] = a0 - a2;
    t[1] = a1 + a2;
    t[2] = a2 - a1;
    t[3] = a1 - a3;
}

// the lane's own columns' B^T from its rows r (rows 0 / 3 masked)
__device__ __forceinline__ void wn_own(const f2v (&r)[4], bool r0ok, bool r3ok, float (&tx)[4],
                                       float (&ty)[4]) {
    wn_bt(r0ok ? r[0].x : 0.f, r[1].x, r[2].x, r3ok ? r[3].x : 0.f, tx);
    wn_bt(r0ok ? r[0].y : 0.f, r[1].y, r[2].y, r3ok ? r[3].y : 0.f, ty);
}

// the outer columns from the neighbour lanes (EDGE: a tile row wider than a
// wave, whose wave-edge lanes transform the neighbour column from memory)
template <bool EDGE>
__device__ __forceinline__ void wn_outer(const float (&tx)[4], const float (&ty)[4],
                                         const float *__restrict__ xc, int ty_, int tx_,
                                         bool r0ok, bool r3ok, int lane, int TW, int H, int W,
                                         float (&tl)[4], float (&tr)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        tl[i] = wn_dpp_left(ty[i]);
        tr[i] = wn_dpp_right(tx[i]);
    }
    if (EDGE) {
        if (lane == 0 && tx_ > 0) {
            float c[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int yy = 2 * ty_ - 1 + i;
                c[i] = (yy >= 0 && yy < H) ? xc[(int64_t)yy * W + 2 * tx_ - 1] : 0.f;
            }
            wn_bt(c[0], c[1], c[2], c[3], tl);
        }
        if (lane == 63 && tx_ < TW - 1) {
            float c[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int yy = 2 * ty_ - 1 + i;
                c[i] = (yy >= 0 && yy < H) ? xc[(int64_t)yy * W + 2 * tx_ + 2] : 0.f;
            }
            wn_bt(c[0], c[1], c[2], c[3], tr);
        }
    }
    (void)r0ok; (void)r3ok;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        tl[i] = tx_ == 0 ? 0.f : tl[i];
        tr[i] = tx_ == TW - 1 ? 0.f : tr[i];
    }
}

// row i of v = t B, t's columns (tl, tx, ty, tr)
__device__ __forceinline__ void wn_vrow(const float (&tl)[4], const float (&tx)[4],
                                        const float (&ty)[4], const float (&tr)[4], int i,
                                        float (&v)[4]) {
    v[0] = tl[i] - ty[i];
    v[1] = tx[i] + ty[i];
    v[2] = ty[i] - tx[i];
    v[3] = tx[i] - tr[i];
}

// one patch row (two floats per lane) at sbase + voff: an ordinary load, so
// the compiler tracks it (an asm load's destination would count as written
// at once, and the compiler may copy or reuse the register before the data
// lands).  Its waits also retire the older filter-stage LDS-DMA (vmcnt is
// in order): safe, at worst early.
// (a buffer load: the base in a uniform descriptor, the lane's 32-bit byte
// offset in one VGPR -- no 64-bit address arithmetic per load)
__device__ __forceinline__ f2v wn_ld2(uint32_t voff, __amdgpu_buffer_rsrc_t rs) {
    return __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 0, 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wn_rsrc(const float *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), 0, 0x7fffffff, 0x00020000);
}

#ifdef WN_CLOCK        // diagnostic build only (-DWN_CLOCK): per-block clock stamps
                       // (tools/wino_pmc.py reads them through smmd_diag_wino_clock)
__device__ unsigned long long wn_clk[4096][4];
// the 8-wave kernel's phases, waves 0 and 4: memtime at entry, after the
// prologue's barrier, after the chunk loop, after the epilogue's two
// barriers, at exit; realtime at entry, exit
__device__ unsigned long long wn_clk8[4096][2][8];
#endif

template <bool EDGE>
__global__ __launch_bounds__(WN_T, 1) void wino_conv_kernel(
    const float *__restrict__ x, const float *__restrict__ u, const float *__restrict__ bias,
    float *__restrict__ y, WnGeom g) {
    extern __shared__ float4 wn_lds[];
    float4 *const Vs = wn_lds;                         // [2][p][h][t64]  (float4 = c4)
    float4 *const Us = wn_lds + 2 * (WN_STAGE / 4);    // [2][p][h][k64]
    float *const Bs = reinterpret_cast<float *>(wn_lds + 4 * (WN_STAGE / 4));   // [k64]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int kb = blockIdx.y;
    const int64_t tile0 = (int64_t)blockIdx.x * WN_TB;
    const int nch1 = g.C / WN_CC;                       // chunks per input
    const int nch = g.x2 ? 2 * nch1 : nch1;             // over both inputs
#ifdef WN_CLOCK
    const unsigned long long clk_t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
    // input-channel slice blockIdx.z of gridDim.z: chunks [c0, c0 + nchunk)
    const int c0 = (int)((int64_t)nch * blockIdx.z / gridDim.z);
    const int nchunk = (int)((int64_t)nch * (blockIdx.z + 1) / gridDim.z) - c0;
    y += (int64_t)blockIdx.z * g.slab;

    // transform role: lane = tile, wave w = channels 2w, 2w+1 of each chunk
    const int64_t gt = tile0 + lane;
    const bool tok = gt < g.T;
    int tn = 0, tty = 0, ttx = 0;
    if (tok) {
        tn = (int)(gt / g.Timg);
        const int r = (int)(gt - (int64_t)tn * g.Timg);
        tty = r / g.TW;
        ttx = r - tty * g.TW;
    }
    const int64_t HW = (int64_t)g.H * g.W;

    // The loop's global loads, all issued at the top of chunk c for chunk
    // c + 1: its filter stage by LDS-DMA (8 asm pieces, no VGPR destination;
    // the compiler does not count them), then its patch rows into `raw` (8
    // ordinary loads, used in this chunk's second half: loaded and used in one
    // iteration, so no loop-carried copy of a register still loading).  The
    // compiler's waits for the rows also retire the older stage pieces (vmcnt
    // is in order); a vmcnt(0) before the barrier makes that explicit.
    // Addresses: a uniform SGPR base per chunk plus fixed per-lane byte
    // offsets (x is under 2 GiB: smmd_wino3x3_supported).
    f2v raw[2][4];
    uint32_t xoff[2][4];                // byte offsets of the rows from the chunk base
    const int TH = g.H >> 1;
    const bool r0ok = tty > 0, r3ok = tty < TH - 1;
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int yc = min(max(2 * tty - 1 + i, 0), g.H - 1);
            xoff[e][i] = (uint32_t)((((int64_t)tn * g.C + 2 * w + e) * HW + (int64_t)yc * g.W +
                                     2 * ttx) * 4);
        }
    // chunk cc of this slice: its input and filter stage (wave-uniform)
    auto xbase = [&](int cc) -> const float * {
        const int c = c0 + cc;
        return c < nch1 ? x + (int64_t)c * WN_CC * HW : g.x2 + (int64_t)(c - nch1) * WN_CC * HW;
    };
    auto ubase = [&](int cc) -> const float4 * {
        const int c = c0 + cc;
        return reinterpret_cast<const float4 *>(c < nch1 ? u : g.u2) +
               ((int64_t)kb * nch1 + (c < nch1 ? c : c - nch1)) * (WN_STAGE / 4);
    };
    auto load_rows = [&](int cc) {
        const __amdgpu_buffer_rsrc_t rs = wn_rsrc(xbase(cc));
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int i = 0; i < 4; ++i) raw[e][i] = wn_ld2(xoff[e][i], rs);
    };
    const uint32_t us_lds = lds_addr(Us) + (uint32_t)__builtin_amdgcn_readfirstlane(w) * 8192u;
    // (per-piece lane offsets, no instruction offset: an LDS-DMA's immediate
    // offset would move its LDS destination too)
    uint32_t uoff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) uoff[i] = (uint32_t)((w * 512 + i * 64 + lane) * 16);
    auto load_u = [&](int cc) {
        const float4 *sb = ubase(cc);
        const uint32_t dst = us_lds + (uint32_t)(cc & 1) * (WN_STAGE * 4);
#pragma unroll
        for (int i = 0; i < 8; ++i) glds16(uoff[i], sb, dst + i * 1024);
    };
    f32x16 acc[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) acc[p] = f32x16{};

    const int th = w & 1, kh = w >> 1, hl = lane >> 5, l32 = lane & 31;
// 64 MFMAs per wave per chunk, the points taken in pairs so consecutive
// MFMAs never share an accumulator; the next pair's fragments are read right
// after each pair's first MFMA (seven MFMAs of cover for the LDS latency)
#define WN_MFMA_CHUNK(BUF_)                                                                  \
    do {                                                                                     \
        const float4 *V_ = Vs + (BUF_) * (WN_STAGE / 4);                                     \
        const float4 *U_ = Us + (BUF_) * (WN_STAGE / 4);                                     \
        float4 a0 = U_[hl * 64 + kh * 32 + l32], b0 = V_[hl * 64 + th * 32 + l32];          \
        float4 a1 = U_[(2 + hl) * 64 + kh * 32 + l32], b1 = V_[(2 + hl) * 64 + th * 32 + l32]; \
        _Pragma("unroll") for (int pp = 0; pp < 8; ++pp) {                                   \
            const int p = 2 * pp;                                                            \
            const float4 ca0 = a0, cb0 = b0, ca1 = a1, cb1 = b1;                             \
            _Pragma("unroll") for (int m = 0; m < 8; ++m) {                                  \
                const int s4 = m >> 1;                                                       \
                if ((m & 1) == 0)                                                            \
                    acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca0[s4], cb0[s4], acc[p], 0, 0, 0); \
                else                                                                         \
                    acc[p + 1] =                                                             \
                        __builtin_amdgcn_mfma_f32_32x32x2f32(ca1[s4], cb1[s4], acc[p + 1], 0, 0, 0); \
                if (m == 0 && pp < 7) {                                                      \
                    a0 = U_[((p + 2) * 2 + hl) * 64 + kh * 32 + l32];                        \
                    b0 = V_[((p + 2) * 2 + hl) * 64 + th * 32 + l32];                        \
                    a1 = U_[((p + 3) * 2 + hl) * 64 + kh * 32 + l32];                        \
                    b1 = V_[((p + 3) * 2 + hl) * 64 + th * 32 + l32];                        \
                }                                                                            \
                __builtin_amdgcn_sched_barrier(0);                                           \
            }                                                                                \
        }                                                                                    \
    } while (0)

    // chunk 0 staged before the loop (everything waited for), chunk 1's rows
    // then issued
    const float bias_k = (bias && tid < WN_KB) ? bias[kb * WN_KB + tid] : 0.f;
    load_u(0);
    load_rows(0);
    {
        float tx[2][4], ty[2][4], tl[4], tr[4], v[2][4][4];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            wn_own(raw[e], r0ok, r3ok, tx[e], ty[e]);
            wn_outer<EDGE>(tx[e], ty[e], xbase(0) + ((int64_t)tn * g.C + 2 * w + e) * HW, tty, ttx,
                           r0ok, r3ok, lane, g.TW, g.H, g.W, tl, tr);
#pragma unroll
            for (int i = 0; i < 4; ++i) wn_vrow(tl, tx[e], ty[e], tr, i, v[e][i]);
        }
        float2 *V2 = reinterpret_cast<float2 *>(Vs);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                V2[(((i * 4 + j) * 2 + (w >> 1)) * 64 + lane) * 2 + (w & 1)] =
                    make_float2(v[0][i][j], v[1][i][j]);
    }
    if (tid < WN_KB) Bs[tid] = bias_k;
    dma_wait_all();                          // chunk 0's stage landed (the rows' waits did it)
    __syncthreads();

    for (int cc = 0; cc + 1 < nchunk; ++cc) {
        const int buf = cc & 1, nbuf = buf ^ 1;
        load_u(cc + 1);
        __builtin_amdgcn_sched_barrier(0);
        load_rows(cc + 1);
        __builtin_amdgcn_sched_barrier(0);
        const float4 *V_ = Vs + buf * (WN_STAGE / 4);
        const float4 *U_ = Us + buf * (WN_STAGE / 4);
        float4 a0 = U_[hl * 64 + kh * 32 + l32], b0 = V_[hl * 64 + th * 32 + l32];
        float4 a1 = U_[(2 + hl) * 64 + kh * 32 + l32], b1 = V_[(2 + hl) * 64 + th * 32 + l32];
        // first half: 32 MFMAs
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
            const int p = 2 * pp;
            const float4 ca0 = a0, cb0 = b0, ca1 = a1, cb1 = b1;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int s4 = m >> 1;
                if ((m & 1) == 0)
                    acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca0[s4], cb0[s4], acc[p], 0, 0, 0);
                else
                    acc[p + 1] =
                        __builtin_amdgcn_mfma_f32_32x32x2f32(ca1[s4], cb1[s4], acc[p + 1], 0, 0, 0);
                if (m == 0) {
                    a0 = U_[((p + 2) * 2 + hl) * 64 + kh * 32 + l32];
                    b0 = V_[((p + 2) * 2 + hl) * 64 + th * 32 + l32];
                    a1 = U_[((p + 3) * 2 + hl) * 64 + kh * 32 + l32];
                    b1 = V_[((p + 3) * 2 + hl) * 64 + th * 32 + l32];
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // second half: after each MFMA one slice of chunk cc + 1's transform
        // and V stores (the other buffer), issued in the MFMA's slot (the f32 MFMA holds the SIMD's VALU, so
        // each slice costs its own issue time); sched_barrier pins the order
        __builtin_amdgcn_sched_barrier(0);
        float tx0[4], ty0[4], tx1[4], ty1[4], tl0[4], tr0[4], tl1[4], tr1[4], v0[4], v1[4];
        const float *xc = xbase(cc + 1) + ((int64_t)tn * g.C + 2 * w) * HW;
        float2 *Vn = reinterpret_cast<float2 *>(Vs + nbuf * (WN_STAGE / 4));
#pragma unroll
        for (int pp = 4; pp < 8; ++pp) {
            const int p = 2 * pp;
            const float4 ca0 = a0, cb0 = b0, ca1 = a1, cb1 = b1;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int s4 = m >> 1;
                if ((m & 1) == 0)
                    acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca0[s4], cb0[s4], acc[p], 0, 0, 0);
                else
                    acc[p + 1] =
                        __builtin_amdgcn_mfma_f32_32x32x2f32(ca1[s4], cb1[s4], acc[p + 1], 0, 0, 0);
                if (m == 0 && pp < 7) {
                    a0 = U_[((p + 2) * 2 + hl) * 64 + kh * 32 + l32];
                    b0 = V_[((p + 2) * 2 + hl) * 64 + th * 32 + l32];
                    a1 = U_[((p + 3) * 2 + hl) * 64 + kh * 32 + l32];
                    b1 = V_[((p + 3) * 2 + hl) * 64 + th * 32 + l32];
                }
                const int K = (pp - 4) * 8 + m;
                // (the rows are first used at slice 8: 40 MFMAs after their
                // loads went out)
                if (K == 8) {                        // own columns, channel 0
                    // (an empty asm on the rows: their arithmetic cannot be
                    // hoisted above this slot, so their wait lands here)
                    asm volatile("" : "+v"(raw[0][0]), "+v"(raw[0][1]), "+v"(raw[0][2]),
                                 "+v"(raw[0][3]), "+v"(raw[1][0]), "+v"(raw[1][1]),
                                 "+v"(raw[1][2]), "+v"(raw[1][3]));
                    wn_own(raw[0], r0ok, r3ok, tx0, ty0);
                } else if (K == 9) {                 // own columns, channel 1
                    wn_own(raw[1], r0ok, r3ok, tx1, ty1);
                } else if (K == 11) {
                    wn_outer<EDGE>(tx0, ty0, xc, tty, ttx, r0ok, r3ok, lane, g.TW, g.H, g.W,
                                   tl0, tr0);
                } else if (K == 13) {
                    wn_outer<EDGE>(tx1, ty1, xc + HW, tty, ttx, r0ok, r3ok, lane, g.TW, g.H, g.W,
                                   tl1, tr1);
                } else if (K >= 16 && K < 20) {      // row i of V, both channels, stored
                    const int i = K - 16;
                    wn_vrow(tl0, tx0, ty0, tr0, i, v0);
                    wn_vrow(tl1, tx1, ty1, tr1, i, v1);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        Vn[(((i * 4 + j) * 2 + (w >> 1)) * 64 + lane) * 2 + (w & 1)] =
                            make_float2(v0[j], v1[j]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        dma_wait_all();                      // chunk cc + 1's filter stage landed
        __syncthreads();
    }
    WN_MFMA_CHUNK((nchunk - 1) & 1);

    // epilogue: C_p[k][tile], k = (r & 3) + 8 (r >> 2) + 4 hl, tile = l32.
    // With an even tile-row width the lane pair (2i, 2i+1) holds two
    // neighbouring tiles: the even lane stores row 0 of both, the odd lane
    // row 1 (one DPP swap of two floats), so every store is a float4
    const int64_t et = tile0 + th * 32 + l32;
    const bool eok = et < g.T;
    const int en = eok ? (int)(et / g.Timg) : 0;
    const int er = (int)(et - (int64_t)en * g.Timg);
    const int ety = er / g.TW, etx = er - ety * g.TW;
    const bool pairs = (g.TW & 1) == 0;
    const bool odd = lane & 1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int k = kb * WN_KB + kh * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        float m[16];
#pragma unroll
        for (int p = 0; p < 16; ++p) m[p] = acc[p][r];
        float s0[4], s1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            s0[j] = m[j] + m[4 + j] + m[8 + j];
            s1[j] = m[4 + j] - m[8 + j] - m[12 + j];
        }
        const float b = Bs[k - kb * WN_KB];
        float y00 = s0[0] + s0[1] + s0[2] + b, y01 = s0[1] - s0[2] - s0[3] + b;
        float y10 = s1[0] + s1[1] + s1[2] + b, y11 = s1[1] - s1[2] - s1[3] + b;
        if (g.relu) {
            y00 = fmaxf(y00, 0.f); y01 = fmaxf(y01, 0.f);
            y10 = fmaxf(y10, 0.f); y11 = fmaxf(y11, 0.f);
        }
        float *o = y + (((int64_t)en * g.K + k) * g.H + 2 * ety) * g.W + 2 * etx;
        if (pairs) {
            // even lanes send row 1, odd lanes row 0, to the partner lane
            const float sx = odd ? y00 : y10, sy = odd ? y01 : y11;
            const float rx = __builtin_bit_cast(
                float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, sx), 0xb1, 0xf, 0xf, false));
            const float ry = __builtin_bit_cast(
                float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, sy), 0xb1, 0xf, 0xf, false));
            if (eok) {
                if (!odd)
                    *reinterpret_cast<float4 *>(o) = make_float4(y00, y01, rx, ry);
                else
                    *reinterpret_cast<float4 *>(o + g.W - 2) = make_float4(rx, ry, y10, y11);
            }
        } else if (eok) {
            *reinterpret_cast<float2 *>(o) = make_float2(y00, y01);
            *reinterpret_cast<float2 *>(o + g.W) = make_float2(y10, y11);
        }
    }
#ifdef WN_CLOCK
    if (tid == 0 && blockIdx.z == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
        const unsigned b = (blockIdx.y * gridDim.x + blockIdx.x) & 4095;
        wn_clk[b][0] = clk_t0; wn_clk[b][1] = t1; wn_clk[b][2] = clk_r0; wn_clk[b][3] = r1;
    }
#endif
}

// The same block tile (64 tiles x 64 output channels, chunks of 8 input
// channels, the same LDS stages) with 8 waves, two per SIMD: waves w and
// w + 4 share a SIMD and the (k, tile) quadrant q = w & 3, and split the 16
// points (PH = w >> 2: points 8 PH .. 8 PH + 7, 128 accumulator registers).
// The f32 MFMA holds its own wave's VALU issue, but the partner wave's VALU
// work goes out beside it (profiles/r12/mfma_valu_coissue.txt: two waves per
// SIMD, the MFMA wave keeps its 64 cycles a slot), so the input transform --
// one channel per wave now -- and the chunk-boundary waits of one wave are
// covered by the other's MFMAs.  Each point's accumulation order over the
// channels is that of wino_conv_kernel and the output transform is its
// arithmetic term for term (the partners swap the halves of their
// accumulators through LDS and each finishes 8 of the 16 rows), so the two
// kernels' outputs are bit-identical.
constexpr int W8_T = 512;
#ifndef W8_VPAIR
#define W8_VPAIR 1      // the V stage in channel pairs (see store_vrow)
#endif
#ifndef W8_VPAD
#define W8_VPAD 1       // each point's V block padded by 8 bytes (see vfrag)
#endif
// floats per point of the 8-wave kernel's V stage, and per V buffer
constexpr int W8_VP = (W8_VPAIR && W8_VPAD) ? 514 : 512;
constexpr int W8_VST = 16 * W8_VP;
static_assert(W8_VST % 4 == 0, "V buffers of whole float4");
static_assert((2 * W8_VST + 2 * WN_STAGE) * sizeof(float) >= 8 * 8 * 2 * 64 * 16,
              "the epilogue's accumulator exchange fits below the biases");

// The 8-wave kernel's transform of one channel where tile rows are whole lane
// groups (no edge loads) and the rows outside the image were loaded as zeros
// (w8 row offsets past the descriptor's range): the column ops on both
// columns packed, and the neighbour columns masked at the SOURCE (a lane at
// its image row's right edge passes 0 to the right neighbour's left column,
// one at the left edge 0 to the left neighbour's right column), so each DPP
// move folds into its subtraction.  Term for term wn_own / wn_outer / wn_vrow.
__device__ __forceinline__ void w8_cols(const f2v (&r)[4], f2v (&t)[4]) {
    t[0] = r[0] - r[2];
    t[1] = r[1] + r[2];
    t[2] = r[2] - r[1];
    t[3] = r[1] - r[3];
}
__device__ __forceinline__ void w8_row(const f2v &t, bool eL, bool eR, float (&v)[4]) {
    const float ys = eR ? 0.f : t.y, xs = eL ? 0.f : t.x;
    v[0] = wn_dpp_left(ys) - t.y;
    v[3] = t.x - wn_dpp_right(xs);
    // (tx + ty, ty - tx) in one packed add: the low result takes (t.lo,
    // t.hi), the high one (t.hi, -t.lo)
    f2v s;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(s) : "v"(t));
    v[1] = s.x;
    v[2] = s.y;
}
#ifndef W8_SLOT
#define W8_SLOT 16      // first MFMA slot of the transform slices (rows issued at the chunk top)
#endif
#ifndef W8_SLOT1
#define W8_SLOT1 W8_SLOT  // the same for the PH = 1 waves
#endif

// The 8-wave kernel's block (tile block, output-channel block, slice) from
// its 1-D id, XCD-aware: blocks b and b + 8 share an XCD and its L2
// (MI355X_MICROARCH.md, dispatch; for speed only, any placement is correct),
// so XCD x takes the x-th contiguous range of the tile-major order ((tile
// block, slice), output-channel block): the output-channel blocks of one
// tile block run together on one L2 and read its x rows once (the 3-D grid
// dealt them to the XCDs round-robin, and each read x again).  Measured and
// not kept: filter-major ((output-channel block, slice), tile block), equal
// on the 512-channel layer, 1-2 % slower on the others
// (profiles/r13/wino8_order_ab.txt).
struct W8Block {
    int64_t tb;
    int kb, sl;
};
__device__ __forceinline__ W8Block w8_block(const WnGeom &g) {
    const uint32_t n = gridDim.x, L = blockIdx.x;
    const uint32_t q = n >> 3, r = n & 7, xc = L & 7, j = L >> 3;
    uint32_t W = xc < r ? xc * (q + 1) + j : r * (q + 1) + (xc - r) * q + j;
    W8Block b;
    b.kb = (int)(W % (uint32_t)g.KB);
    W /= (uint32_t)g.KB;
    b.sl = (int)(W % (uint32_t)g.S);
    b.tb = W / (uint32_t)g.S;
    return b;
}

template <bool EDGE, int PH, int EPI>
__device__ __forceinline__ void wino8_body(const float *__restrict__ x, const float *__restrict__ u,
                                           const float *__restrict__ bias, float *__restrict__ y,
                                           const WnGeom &g) {
    extern __shared__ float4 wn_lds[];
    float4 *const Vs = wn_lds;                         // [2][p][h][cp][t64][c2] (see store_vrow)
    float4 *const Us = wn_lds + 2 * (W8_VST / 4);      // [2][p][h][k64]
    float *const Bs = reinterpret_cast<float *>(Us + 2 * (WN_STAGE / 4));   // [k64]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const W8Block blk = w8_block(g);
    const int kb = blk.kb;
    const int64_t tile0 = blk.tb * WN_TB;
    const int nch1 = g.C / WN_CC;
    const int nch = g.x2 ? 2 * nch1 : nch1;
    const int c0 = (int)((int64_t)nch * blk.sl / g.S);
    const int nchunk = (int)((int64_t)nch * (blk.sl + 1) / g.S) - c0;
    y += (int64_t)blk.sl * g.slab;
#ifdef WN_CLOCK
    unsigned long long ck[8];
    ck[0] = __builtin_amdgcn_s_memtime();
    ck[6] = __builtin_amdgcn_s_memrealtime();
#endif

    // transform role: lane = tile, wave w = channel w of each chunk
    const int64_t gt = tile0 + lane;
    const bool tok = gt < g.T;
    int tn = 0, tty = 0, ttx = 0;
    if (tok) {
        tn = (int)(gt / g.Timg);
        const int r = (int)(gt - (int64_t)tn * g.Timg);
        tty = r / g.TW;
        ttx = r - tty * g.TW;
    }
    const int64_t HW = (int64_t)g.H * g.W;
    f2v raw[4];
    uint32_t xoff[4];
    const int TH = g.H >> 1;
    const bool r0ok = tty > 0, r3ok = tty < TH - 1;
    // (a row outside the image: an offset past the descriptor's range, so
    // the load returns zeros)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int yy = 2 * tty - 1 + i;
        xoff[i] = (yy < 0 || yy >= g.H)
                      ? 0x80000000u
                      : (uint32_t)((((int64_t)tn * g.C + w) * HW + (int64_t)yy * g.W + 2 * ttx) * 4);
    }
    const bool eL = ttx == 0, eR = ttx == g.TW - 1;
    auto xbase = [&](int cc) -> const float * {
        const int c = c0 + cc;
        return c < nch1 ? x + (int64_t)c * WN_CC * HW : g.x2 + (int64_t)(c - nch1) * WN_CC * HW;
    };
    auto ubase = [&](int cc) -> const float4 * {
        const int c = c0 + cc;
        return reinterpret_cast<const float4 *>(c < nch1 ? u : g.u2) +
               ((int64_t)kb * nch1 + (c < nch1 ? c : c - nch1)) * (WN_STAGE / 4);
    };
    auto load_rows = [&](int cc) {
        const __amdgpu_buffer_rsrc_t rs = wn_rsrc(xbase(cc));
#pragma unroll
        for (int i = 0; i < 4; ++i) raw[i] = wn_ld2(xoff[i], rs);
    };
    // filter stage: 4 LDS-DMA pieces per wave
    const uint32_t us_lds = lds_addr(Us) + (uint32_t)__builtin_amdgcn_readfirstlane(w) * 4096u;
    uint32_t uoff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) uoff[i] = (uint32_t)((w * 256 + i * 64 + lane) * 16);
    auto load_u = [&](int cc) {
        const float4 *sb = ubase(cc);
        const uint32_t dst = us_lds + (uint32_t)(cc & 1) * (WN_STAGE * 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) glds16(uoff[i], sb, dst + i * 1024);
    };
    // V of this wave's channel (h = w >> 2, c4 = w & 3).  W8_VPAIR (default):
    // float index ((((p h) cp) t) c2) with cp = c4 >> 1, c2 = c4 & 1 -- a
    // wave's ds_write_b32 then covers 16 banks of the 32 (2-way: no cost;
    // the [t][c4] form's 4-way conflict doubled every V store) and a fragment
    // is two conflict-free ds_read_b64 (the same 4 cycles as one b128);
    // otherwise ((p h t) c4).  The MFMA operands are the same registers.
#if W8_VPAIR
    const int vlane = (((w >> 2) * 2 + ((w & 3) >> 1)) * 64 + lane) * 2 + (w & 1);
#endif
    auto store_vrow = [&](float *Vf, int i, const float (&v)[4]) {
#ifdef W8_NO_VSTORE       // timing-only diagnostic: the transform kept, its stores not issued
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(v[j]));
        return;
#endif
#pragma unroll
        for (int j = 0; j < 4; ++j)
#if W8_VPAIR
            (Vf + vlane)[(i * 4 + j) * W8_VP] = v[j];
#else
            Vf[(((i * 4 + j) * 2 + (w >> 2)) * 64 + lane) * 4 + (w & 3)] = v[j];
#endif
    };
    f32x16 acc[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p] = f32x16{};

    const int q = w & 3, th = q & 1, kh = q >> 1, hl = lane >> 5, l32 = lane & 31;
    // a V fragment (point p, this lane's reduction half and tile)
#if W8_VPAIR
    // the channel pair's second half 64 f2v on, through an opaque (uniform)
    // offset: two ds_read_b64 (4 cycles), not one merged ds_read2_b64 (8)
    int vhi;
    asm volatile("s_mov_b32 %0, 64" : "=s"(vhi));
#endif
    auto vfrag = [&](const float4 *V_, int p) -> float4 {
#if W8_VPAIR
        const f2v *V2 = reinterpret_cast<const f2v *>(V_) + (hl * 2 * 64 + th * 32 + l32);
        // (W8_VPAD: a point's block is W8_VP = 514 floats, 2056 B, so the
        // reads of points p and p + 1 are no pair the compiler can merge into
        // one ds_read2st64_b64, 8 cycles, against two ds_read_b64 of 2 each)
        const f2v lo = V2[p * (W8_VP / 2)];
        const f2v hi = (V2 + vhi)[p * (W8_VP / 2)];
        return float4{lo.x, lo.y, hi.x, hi.y};
#else
        return V_[(p * 2 + hl) * 64 + th * 32 + l32];
#endif
    };
    constexpr int P0 = 8 * PH;
    constexpr int SL = PH ? W8_SLOT1 : W8_SLOT;
    const float bias_k = (bias && tid < WN_KB) ? bias[kb * WN_KB + tid] : 0.f;
    load_u(0);
    load_rows(0);
    if constexpr (EDGE) {
        float tx[4], ty[4], tl[4], tr[4], v[4];
        wn_own(raw, r0ok, r3ok, tx, ty);
        wn_outer<EDGE>(tx, ty, xbase(0) + ((int64_t)tn * g.C + w) * HW, tty, ttx, r0ok, r3ok, lane,
                       g.TW, g.H, g.W, tl, tr);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            wn_vrow(tl, tx, ty, tr, i, v);
            store_vrow(reinterpret_cast<float *>(Vs), i, v);
        }
    } else {
        f2v t[4];
        float v[4];
        w8_cols(raw, t);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            w8_row(t[i], eL, eR, v);
            store_vrow(reinterpret_cast<float *>(Vs), i, v);
        }
    }
    if (tid < WN_KB) Bs[tid] = bias_k;
    dma_wait_all();
    __syncthreads();
#ifdef WN_CLOCK
    ck[1] = __builtin_amdgcn_s_memtime();
#endif

    for (int cc = 0;; ++cc) {
        const bool more = cc + 1 < nchunk;
        const int buf = cc & 1, nbuf = buf ^ 1;
        // the first fragments' LDS reads go out first, so their latency runs
        // under the next chunk's load issue
        const float4 *V_ = Vs + buf * (W8_VST / 4);
        const float4 *U_ = Us + buf * (WN_STAGE / 4);
        float4 a0 = U_[(P0 * 2 + hl) * 64 + kh * 32 + l32], b0 = vfrag(V_, P0);
        float4 a1 = U_[((P0 + 1) * 2 + hl) * 64 + kh * 32 + l32], b1 = vfrag(V_, P0 + 1);
        __builtin_amdgcn_sched_barrier(0);
        if (more) {
#ifndef W8_NO_DMA         // (W8_NO_*: timing-only diagnostic builds, wrong results)
            load_u(cc + 1);
#endif
            __builtin_amdgcn_sched_barrier(0);
#ifndef W8_NO_ROWS
            load_rows(cc + 1);
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
        float tx[4], ty[4], tl[4], tr[4], v[4];
        f2v t[4];
        const float *xc = more ? xbase(cc + 1) + ((int64_t)tn * g.C + w) * HW : x;
        float *Vn = reinterpret_cast<float *>(Vs + nbuf * (W8_VST / 4));
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
            const int p = P0 + 2 * pp;
            const float4 ca0 = a0, cb0 = b0, ca1 = a1, cb1 = b1;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int s4 = m >> 1;
                if ((m & 1) == 0)
                    acc[2 * pp] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca0[s4], cb0[s4], acc[2 * pp], 0, 0, 0);
                else
                    acc[2 * pp + 1] =
                        __builtin_amdgcn_mfma_f32_32x32x2f32(ca1[s4], cb1[s4], acc[2 * pp + 1], 0, 0, 0);
                if (m == 0 && pp < 3) {
                    a0 = U_[((p + 2) * 2 + hl) * 64 + kh * 32 + l32];
                    b0 = vfrag(V_, p + 2);
                    a1 = U_[((p + 3) * 2 + hl) * 64 + kh * 32 + l32];
                    b1 = vfrag(V_, p + 3);
                }
                const int K = pp * 8 + m;
#ifdef W8_NO_XFORM
                if (false) {
#else
                if (more) {
#endif
                    if (K == SL) {
                        asm volatile("" : "+v"(raw[0]), "+v"(raw[1]), "+v"(raw[2]), "+v"(raw[3]));
                        if constexpr (EDGE)
                            wn_own(raw, r0ok, r3ok, tx, ty);
                        else
                            w8_cols(raw, t);
                    } else if (EDGE && K == SL + 2) {
                        wn_outer<EDGE>(tx, ty, xc, tty, ttx, r0ok, r3ok, lane, g.TW, g.H, g.W, tl,
                                       tr);
                    } else if (K >= SL + 4 && K < SL + 8) {
                        if constexpr (EDGE)
                            wn_vrow(tl, tx, ty, tr, K - SL - 4, v);
                        else
                            w8_row(t[K - SL - 4], eL, eR, v);
                        store_vrow(Vn, K - SL - 4, v);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (!more) break;
        dma_wait_all();
        __syncthreads();
    }
#ifdef WN_CLOCK
    ck[2] = __builtin_amdgcn_s_memtime();
#endif

    // epilogue: the partners swap accumulator halves (rows 8 (1 - PH) ..
    // through LDS, the stages being free once every wave is past its last
    // MFMA), then each finishes rows 8 PH .. 8 PH + 7 of the quadrant with all
    // 16 points.  X[w][p local][r4][lane] float4 (16 KB per wave).
    const int partner = w ^ 4;
    const int64_t et = tile0 + th * 32 + l32;
    const bool eok = et < g.T;
    const int en = eok ? (int)(et / g.Timg) : 0;
    const int er = (int)(et - (int64_t)en * g.Timg);
    const int ety = er / g.TW, etx = er - ety * g.TW;
    const int k0 = kb * WN_KB + kh * 32 + 4 * hl;
    const uint32_t yo =
        (uint32_t)(((((int64_t)en * g.K + k0) * g.H + 2 * ety) * g.W + 2 * etx) * 4);
    const uint32_t hw4 = (uint32_t)(HW * 4), yo1 = yo + (uint32_t)g.W * 4;
    // EPI 2: the mask's 32 values of the lane, loaded before the exchange (a
    // tile past the end reads zeros at the out-of-range offset and is not stored)
    f2v mk[2][2][2][2];
    if constexpr (EPI == 2) {
        const __amdgpu_buffer_rsrc_t ms = wn_rsrc(g.mask);
        const uint32_t m0 = eok ? yo : 0x80000000u, m1 = eok ? yo1 : 0x80000000u;
#pragma unroll
        for (int r4 = 0; r4 < 2; ++r4)
#pragma unroll
            for (int rp = 0; rp < 2; ++rp) {
                const int r = 8 * PH + 4 * r4 + 2 * rp;
                const int kr = (r & 3) + 8 * (r >> 2);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t so = (uint32_t)(kr + h) * hw4;
                    mk[r4][rp][h][0] = __builtin_bit_cast(
                        f2v, __builtin_amdgcn_raw_buffer_load_b64(ms, m0, so, 0));
                    mk[r4][rp][h][1] = __builtin_bit_cast(
                        f2v, __builtin_amdgcn_raw_buffer_load_b64(ms, m1, so, 0));
                }
            }
    }
    __syncthreads();
#ifdef WN_CLOCK
    ck[3] = __builtin_amdgcn_s_memtime();
#endif
    float4 *const X = wn_lds;
    constexpr int RO = 8 * (1 - PH);       // rows handed to the partner
#pragma unroll
    for (int p = 0; p < 8; ++p)
#pragma unroll
        for (int r4 = 0; r4 < 2; ++r4)
            X[((w * 8 + p) * 2 + r4) * 64 + lane] =
                make_float4(acc[p][RO + 4 * r4], acc[p][RO + 4 * r4 + 1], acc[p][RO + 4 * r4 + 2],
                            acc[p][RO + 4 * r4 + 3]);
    __syncthreads();
#ifdef WN_CLOCK
    ck[4] = __builtin_amdgcn_s_memtime();
#endif
    // stores: a uniform descriptor on this slab, the lane's byte offset of
    // its row-0 channel (k0) fixed, each row adding a uniform multiple of H W
    // (y under 2 GiB: smmd_wino3x3_supported); each lane stores its own
    // tile's two output rows (8 bytes each, 32 tiles of a row contiguous)
    const __amdgpu_buffer_rsrc_t ys = wn_rsrc(y);
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    // the output transform on row pairs (r, r + 1): both rows' values of a
    // point sit in adjacent registers (acc[p][r], acc[p][r + 1]; the
    // partner's float4), so every add is one packed op on the pair
#pragma unroll
    for (int r4 = 0; r4 < 2; ++r4) {
        float4 o4[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) o4[p] = X[((partner * 8 + p) * 2 + r4) * 64 + lane];
#pragma unroll
        for (int rp = 0; rp < 2; ++rp) {
            const int r = 8 * PH + 4 * r4 + 2 * rp;           // even: rows r, r + 1 -> k, k + 1
            const int kr = (r & 3) + 8 * (r >> 2);            // k - k0 of row r
            f2v m[16];
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                m[P0 + p] = f2v{acc[p][r], acc[p][r + 1]};
                m[8 - P0 + p] = rp ? f2v{o4[p].z, o4[p].w} : f2v{o4[p].x, o4[p].y};
            }
            f2v s0[4], s1[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                s0[j] = m[j] + m[4 + j] + m[8 + j];
                s1[j] = m[4 + j] - m[8 + j] - m[12 + j];
            }
            const f2v b = *reinterpret_cast<const f2v *>(Bs + (k0 - kb * WN_KB) + kr);
            f2v y00 = s0[0] + s0[1] + s0[2] + b, y01 = s0[1] - s0[2] - s0[3] + b;
            f2v y10 = s1[0] + s1[1] + s1[2] + b, y11 = s1[1] - s1[2] - s1[3] + b;
            if constexpr (EPI == 1) {
                y00 = __builtin_elementwise_max(y00, f2v{0.f, 0.f});
                y01 = __builtin_elementwise_max(y01, f2v{0.f, 0.f});
                y10 = __builtin_elementwise_max(y10, f2v{0.f, 0.f});
                y11 = __builtin_elementwise_max(y11, f2v{0.f, 0.f});
            }
            if (eok) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t so = (uint32_t)(kr + h) * hw4;
                    if constexpr (EPI == 2) {     // row 2 ety: (y00, y01), row + 1: (y10, y11)
                        const f2v a = mk[r4][rp][h][0], c = mk[r4][rp][h][1];
                        y00[h] = a.x <= 0.f ? 0.f : y00[h];
                        y01[h] = a.y <= 0.f ? 0.f : y01[h];
                        y10[h] = c.x <= 0.f ? 0.f : y10[h];
                        y11[h] = c.y <= 0.f ? 0.f : y11[h];
                    }
                    __builtin_amdgcn_raw_buffer_store_b64(
                        __builtin_bit_cast(u2v, f2v{y00[h], y01[h]}), ys, yo, so, 0);
                    __builtin_amdgcn_raw_buffer_store_b64(
                        __builtin_bit_cast(u2v, f2v{y10[h], y11[h]}), ys, yo1, so, 0);
                }
            }
        }
    }
#ifdef WN_CLOCK
    ck[5] = __builtin_amdgcn_s_memtime();
    ck[7] = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && (w & 3) == 0 && blk.sl == 0) {
        const unsigned b = (unsigned)(kb * g.TB + blk.tb) & 4095;
        for (int i = 0; i < 8; ++i) wn_clk8[b][PH][i] = ck[i];
    }
#endif
}

template <bool EDGE, int EPI>
__global__ __launch_bounds__(W8_T, 1) void wino_conv8_kernel(
    const float *__restrict__ x, const float *__restrict__ u, const float *__restrict__ bias,
    float *__restrict__ y, WnGeom g) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 8))
        wino8_body<EDGE, 1, EPI>(x, u, bias, y, g);
    else
        wino8_body<EDGE, 0, EPI>(x, u, bias, y, g);
}

// y = bias + sum over the S partial slabs in slice order (float4 when the
// plane size allows)
__global__ void wino_reduce_kernel(const float *__restrict__ part, const float *__restrict__ bias,
                                   float *__restrict__ y, int64_t n4, int S, int K, int HW,
                                   int relu, const float *__restrict__ mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const float4 *p4 = reinterpret_cast<const float4 *>(part);
    float4 s = p4[i];
    for (int z = 1; z < S; ++z) {
        const float4 t = p4[i + z * n4];
        s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    if (bias) {
        const float b = bias[(int)((i * 4 / HW) % K)];
        s.x += b; s.y += b; s.z += b; s.w += b;
    }
    if (relu == 1) {
        s.x = fmaxf(s.x, 0.f); s.y = fmaxf(s.y, 0.f); s.z = fmaxf(s.z, 0.f); s.w = fmaxf(s.w, 0.f);
    } else if (relu == 2) {
        const float4 m = reinterpret_cast<const float4 *>(mask)[i];
        s.x = m.x <= 0.f ? 0.f : s.x;
        s.y = m.y <= 0.f ? 0.f : s.y;
        s.z = m.z <= 0.f ? 0.f : s.z;
        s.w = m.w <= 0.f ? 0.f : s.w;
    }
    reinterpret_cast<float4 *>(y)[i] = s;
}

}  // namespace

// input-channel slices for a grid of `blocks` workgroups: enough for one
// workgroup per CU, at least 4 chunks (32 channels) per slice (measured on the
// 512-channel 8 x 8 layer: 128 workgroups 183 us, 4 slices 115 us; on the
// 256-channel 16 x 16 one, 256 workgroups, 2 slices 115 us vs none 100 us)
static int wino_slices(int64_t blocks, int nch, int HW) {
    int S = 1;
    while (blocks * S < 256 && nch / (2 * S) >= 4 && HW % 4 == 0) S *= 2;
    return S;
}

// SMMD_WINO8=0: the 4-wave form (A/B and tests; the two are bit-identical)
static bool wino8_enabled() {
    const char *e = getenv("SMMD_WINO8");
    return !(e && e[0] == '0');
}

}  // namespace smmd

using namespace smmd;

#ifdef WN_CLOCK
extern "C" int smmd_diag_wino_clock(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(wn_clk), sizeof(unsigned long long) * 4 * n) ==
                   hipSuccess ? 0 : 1;
}
extern "C" int smmd_diag_wino8_clock(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(wn_clk8), sizeof(unsigned long long) * 16 * n) ==
                   hipSuccess ? 0 : 1;
}
#endif

extern "C" size_t smmd_wino3x3_filter_bytes(int ko, int ci) {
    if (ko <= 0 || ci <= 0) return 0;
    return (size_t)16 * ko * ci * sizeof(float);
}

// (x and y under 2 GiB: the conv kernels address them by 32-bit byte offsets
// into a buffer range of 0x7fffffff bytes, and an offset at or past 2^31 is
// the out-of-range sentinel that reads zeros)
extern "C" int smmd_wino3x3_supported(int n, int ci, int ko, int h, int w_img) {
    return n > 0 && ci > 0 && ko > 0 && ci % WN_CC == 0 && ko % WN_KB == 0 && h > 0 &&
           w_img > 0 && h % 2 == 0 && w_img % 2 == 0 && (int64_t)n * ci * h * w_img < (1ll << 29) &&
           (int64_t)n * ko * h * w_img < (1ll << 29);
}

extern "C" smmd_status smmd_wino3x3_filter(const float *w, int ko, int ci, int mode, float *u,
                                           size_t u_bytes, smmd_stream_t stream) {
    if (ko <= 0 || ci <= 0 || (mode != 0 && mode != 1) || !w || !u) return SMMD_EINVAL;
    if (ko % WN_KB || ci % WN_CC) return SMMD_EUNSUPPORTED;
    if (reinterpret_cast<uintptr_t>(u) & 15) return SMMD_EINVAL;
    if (u_bytes < smmd_wino3x3_filter_bytes(ko, ci)) return SMMD_EWORKSPACE;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t n = (int64_t)ko * (ci / 4);
    wino_filter_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(w, ko, ci, mode, u,
                                                                               nullptr, nullptr);
    return last_launch_status();
}

extern "C" smmd_status smmd_wino3x3_filter_sn(const float *w, const float *sigma, const float *s,
                                              int ko, int ci, int mode, float *u, size_t u_bytes,
                                              smmd_stream_t stream) {
    if (ko <= 0 || ci <= 0 || (mode != 0 && mode != 1) || !w || !u || !sigma) return SMMD_EINVAL;
    if (ko % WN_KB || ci % WN_CC) return SMMD_EUNSUPPORTED;
    if (reinterpret_cast<uintptr_t>(u) & 15) return SMMD_EINVAL;
    if (u_bytes < smmd_wino3x3_filter_bytes(ko, ci)) return SMMD_EWORKSPACE;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t n = (int64_t)ko * (ci / 4);
    wino_filter_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(w, ko, ci, mode, u,
                                                                               sigma, s);
    return last_launch_status();
}

extern "C" size_t smmd_wino3x3_workspace_bytes(int n, int ci, int ko, int h, int w_img) {
    if (!smmd_wino3x3_supported(n, ci, ko, h, w_img)) return 0;
    const int64_t T = (int64_t)n * (h / 2) * (w_img / 2);
    const int S = wino_slices(((T + WN_TB - 1) / WN_TB) * (ko / WN_KB), ci / WN_CC, h * w_img);
    return S > 1 ? (size_t)S * n * ko * h * w_img * sizeof(float) : 0;
}

static smmd_status wino3x3_conv(const float *x, const float *u, const float *x2,
                                const float *u2, const float *bias, float *y, int n, int ci,
                                int ko, int h, int w_img, void *ws, size_t ws_bytes, int relu,
                                smmd_stream_t stream, const float *mask = nullptr) {
    if (n < 0 || ci <= 0 || ko <= 0 || h < 0 || w_img < 0) return SMMD_EINVAL;
    if (n == 0 || h == 0 || w_img == 0) return SMMD_OK;
    if (!x || !u || !y || (!x2 != !u2) || ((relu == 2) != (mask != nullptr))) return SMMD_EINVAL;
    if (!smmd_wino3x3_supported(n, ci, ko, h, w_img)) return SMMD_EUNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
         reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(x2) |
         reinterpret_cast<uintptr_t>(u2) | reinterpret_cast<uintptr_t>(mask)) & 15)
        return SMMD_EINVAL;
    // the mask epilogue is the 8-wave kernel's (the 4-wave form: unsupported)
    if (relu == 2 && !wino8_enabled()) return SMMD_EUNSUPPORTED;
    const int pair = x2 ? 2 : 1;
    WnGeom g;
    g.mask = mask;
    g.x2 = x2;
    g.u2 = u2;
    g.N = n; g.C = ci; g.K = ko; g.H = h; g.W = w_img;
    g.TW = w_img / 2;
    g.Timg = (h / 2) * g.TW;
    g.T = (int64_t)n * g.Timg;
    const int64_t tb = (g.T + WN_TB - 1) / WN_TB;
    if (tb > 0x7fffffff) return SMMD_EINVAL;
    const int S = wino_slices(tb * (ko / WN_KB), pair * ci / WN_CC, h * w_img);
    const int64_t total = (int64_t)n * ko * h * w_img;
    float *out = y;
    if (S > 1) {
        if (!ws || ws_bytes < (size_t)S * total * sizeof(float)) return SMMD_EWORKSPACE;
        if (reinterpret_cast<uintptr_t>(ws) & 15) return SMMD_EINVAL;
        out = static_cast<float *>(ws);
    }
    static bool attr = false;
    if (!attr) {
        const void *ks[8] = {reinterpret_cast<const void *>(wino_conv_kernel<false>),
                             reinterpret_cast<const void *>(wino_conv_kernel<true>),
                             reinterpret_cast<const void *>(wino_conv8_kernel<false, 0>),
                             reinterpret_cast<const void *>(wino_conv8_kernel<true, 0>),
                             reinterpret_cast<const void *>(wino_conv8_kernel<false, 1>),
                             reinterpret_cast<const void *>(wino_conv8_kernel<true, 1>),
                             reinterpret_cast<const void *>(wino_conv8_kernel<false, 2>),
                             reinterpret_cast<const void *>(wino_conv8_kernel<true, 2>)};
        for (const void *k : ks)
            if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WN_LDS) !=
                hipSuccess)
                return SMMD_EHIP;
        attr = true;
    }
    g.slab = S > 1 ? total : 0;
    g.relu = S > 1 ? 0 : relu;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)tb, (unsigned)(ko / WN_KB), (unsigned)S);
    const float *b1 = S > 1 ? nullptr : bias;
    // tile rows that are whole lane groups of a wave need no edge loads
    const bool edge = 64 % g.TW != 0;
    if (wino8_enabled()) {
        g.TB = (int)tb;
        g.KB = ko / WN_KB;
        g.S = S;
        const int64_t nblk = tb * g.KB * S;
        if (nblk > 0x7fffffff) return SMMD_EINVAL;
        auto k8 = edge ? (g.relu == 2   ? wino_conv8_kernel<true, 2>
                          : g.relu ? wino_conv8_kernel<true, 1>
                                   : wino_conv8_kernel<true, 0>)
                       : (g.relu == 2   ? wino_conv8_kernel<false, 2>
                          : g.relu ? wino_conv8_kernel<false, 1>
                                   : wino_conv8_kernel<false, 0>);
        k8<<<dim3((unsigned)nblk), dim3(W8_T), WN_LDS, st>>>(x, u, b1, out, g);
    } else if (!edge) {
        wino_conv_kernel<false><<<grid, dim3(WN_T), WN_LDS, st>>>(x, u, b1, out, g);
    } else {
        wino_conv_kernel<true><<<grid, dim3(WN_T), WN_LDS, st>>>(x, u, b1, out, g);
    }
    smmd_status e = last_launch_status();
    if (e != SMMD_OK || S == 1) return e;
    const int64_t n4 = total / 4;
    wino_reduce_kernel<<<dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st>>>(
        out, bias, y, n4, S, ko, h * w_img, relu, mask);
    return last_launch_status();
}

extern "C" smmd_status smmd_wino3x3_conv(const float *x, const float *u, const float *bias,
                                         float *y, int n, int ci, int ko, int h, int w_img,
                                         void *ws, size_t ws_bytes, smmd_stream_t stream) {
    return wino3x3_conv(x, u, nullptr, nullptr, bias, y, n, ci, ko, h, w_img, ws, ws_bytes, 0,
                        stream);
}

extern "C" size_t smmd_wino3x3_conv2_workspace_bytes(int n, int ci, int ko, int h, int w_img) {
    if (!smmd_wino3x3_supported(n, ci, ko, h, w_img)) return 0;
    const int64_t T = (int64_t)n * (h / 2) * (w_img / 2);
    const int S = wino_slices(((T + WN_TB - 1) / WN_TB) * (ko / WN_KB), 2 * ci / WN_CC, h * w_img);
    return S > 1 ? (size_t)S * n * ko * h * w_img * sizeof(float) : 0;
}

extern "C" smmd_status smmd_wino3x3_conv2(const float *x, const float *u, const float *x2,
                                          const float *u2, const float *bias, float *y, int n,
                                          int ci, int ko, int h, int w_img, void *ws,
                                          size_t ws_bytes, smmd_stream_t stream) {
    if (!x2 || !u2) return SMMD_EINVAL;
    return wino3x3_conv(x, u, x2, u2, bias, y, n, ci, ko, h, w_img, ws, ws_bytes, 0, stream);
}

extern "C" smmd_status smmd_wino3x3_conv_relu(const float *x, const float *u, const float *bias,
                                              float *y, int n, int ci, int ko, int h, int w_img,
                                              void *ws, size_t ws_bytes, smmd_stream_t stream) {
    return wino3x3_conv(x, u, nullptr, nullptr, bias, y, n, ci, ko, h, w_img, ws, ws_bytes, 1,
                        stream);
}

// y = (mask <= 0 ? 0 : conv(x, U) + bias), mask of y's shape: the input
// gradient's ReLU mask of the next layer applied in the epilogue (convops
// _ConvBackward's gy_mask: the double backward's upstream gradient of a
// conv-ReLU whose consumer masks)
extern "C" smmd_status smmd_wino3x3_conv_mask(const float *x, const float *u, const float *bias,
                                              const float *mask, float *y, int n, int ci, int ko,
                                              int h, int w_img, void *ws, size_t ws_bytes,
                                              smmd_stream_t stream) {
    if (!mask) return SMMD_EINVAL;
    return wino3x3_conv(x, u, nullptr, nullptr, bias, y, n, ci, ko, h, w_img, ws, ws_bytes, 2,
                        stream, mask);
}
