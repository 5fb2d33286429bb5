// smmd_conv1x1.hip -- the 1x1 convolutions of the residual blocks' shortcuts
// (gan/core/resnet/block.py:28-40: MeanPoolConv in the critic's down blocks,
// the 1x1 conv before the nearest upsample in the generator's up blocks) on
// the f32 MFMA, NCHW in place: no layout transposes.
//
// All three directions are GEMMs over a "column" index j = (n, p) of the
// batch and the pixels (p fastest, images stride M P):
//   forward          y[n][k][p]  = sum_c W[k][c] x[n][c][p] (+ b[k])
//   input gradient   dx[n][c][p] = sum_k W[k][c] gy[n][k][p]  (the forward with
//                    A = W^T, a [C][K] copy the caller keeps per weight)
//   weight gradient  dW[k][c]    = sum_{n,p} gy[n][k][p] x[n][c][p]
// MIOpen ran them through NHWC transposes (batched_transpose) and igemm /
// GEMM solvers at 15-45 us per 1.07 GFLOP call; the step spent ~8 % of its GPU
// time there (profiles/r14/step_kernel_top_r14g.txt).
//
// c1_gemm (forward / input gradient): block = 64 rows m x 64 columns j, 4 waves,
// wave (mh, jh) the 32 x 32 quadrant on v_mfma_f32_32x32x2_f32.  The reduction
// runs in chunks of 32 through a double-buffered LDS stage kept in the global
// layouts: A [m][r] (row stride 36), B [r][j] (row stride 68), both with
// 16-byte rows for the float4 stores.  MFMA t of a chunk reduces over r = t
// and 16 + t (lane half h = lane / 32 takes 16 h + t): a lane's A values are
// one contiguous run (a 16-byte read feeds 4 MFMAs), its B values one read
// per MFMA (pairs merged into ds_read2_b32).  The next chunk's
// global loads (float4 along the contiguous dimension) are issued before the
// current chunk's MFMAs and stored to the other buffer after them; occupancy
// (4 blocks per CU) covers the rest.
//
// c1_wgrad: block = 64 k x 64 c over one slice of the columns; A = gy [k][j],
// B = x [c][j], both [row][j] with row stride 36 and the same t / 16 + t
// pairing (one 16-byte read of each feeds 4 MFMAs), chunks of 32 columns; each
// slice writes a partial dW, the slices are added in order by c1_sum.
//
// Accumulation order: fixed (per chunk, MFMA t in order; slices in order), so
// the results are deterministic; fp32 products and sums, as the reference.
#include "smmd_common.hpp"
#include "smmd_ldsdma.hpp"

namespace smmd {

namespace {

constexpr int C1_T = 256;
constexpr int C1_RC = 32;                   // reduction values per chunk
constexpr int C1_AS = C1_RC + 4;            // [row][32] stage row stride: 16-byte rows
constexpr int C1_BS = 64 + 4;               // B row stride (floats)
constexpr int C1_ASTAGE = 64 * C1_AS;
constexpr int C1_BSTAGE = C1_RC * C1_BS;
constexpr int C1_STAGE = C1_ASTAGE + C1_BSTAGE;
constexpr int C1_WS = 64 * C1_AS;           // wgrad stage per operand: 64 rows x 36

typedef float f32x16 __attribute__((ext_vector_type(16)));

// column j of an [N][rows][P] tensor: byte-free float offset of (row, j)
__device__ __forceinline__ int64_t c1_off(int64_t j, int row, int rows, int P) {
    const int64_t n = j / P;
    const int64_t p = j - n * P;
    return (n * rows + row) * (int64_t)P + p;
}

// forward / input gradient: Y [N][M][P] = A [M][R] . X [N][R][P] (+ bias[m])
// Split-K: blockIdx.y = slice s of the reduction, chunks [s cps, (s + 1) cps)
// of 32; with several slices Y is slab s of the workspace (bias NULL) and
// c1_sum adds the slabs in order.  TA: A given as its transpose, [R][M] (the
// input gradient straight from W [K][C]: no per-step W^T copy); the thread's
// float4 runs along m and goes to the [m][r] stage as four scalar stores.
template <bool TA>
__global__ __launch_bounds__(C1_T) void c1_gemm_kernel(const float *__restrict__ A,
                                                       const float *__restrict__ X,
                                                       const float *__restrict__ bias,
                                                       float *__restrict__ Y, int M, int R, int P,
                                                       int64_t J, int cps) {
    __shared__ float lds[2 * C1_STAGE];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // blocks: the row blocks of one column tile run on one XCD (its X
    // columns, the large operand, read once into that L2)
    const int mb_n = M / 64;
    const int64_t jb_n = J / 64;
    const int64_t blk = xcd_order(blockIdx.x, (int)(jb_n * mb_n));
    const int mb = (int)(blk % mb_n);
    const int64_t jb = blk / mb_n;
    const int m0 = mb * 64;
    const int64_t j0 = jb * 64;

    // global -> register loads of one chunk: A 64 x 32 (2 float4 / thread,
    // thread -> (row f / 8, quad f % 8)), X 32 x 64 (2 float4 / thread,
    // thread -> (row f / 16, quad f % 16)); the thread's element offsets at
    // chunk 0 (chunk c adds 32 c to A's and 32 c P to X's): the (n, p) split
    // of its columns is done once.
    const int f0 = tid, f1 = tid + C1_T;
    const int rbeg = blockIdx.y * cps * C1_RC;
    const int nchunk = min(cps, R / C1_RC - (int)blockIdx.y * cps);
    // (TA: thread -> row r = (f & 7) + 8 (f >> 7) of A^T, quad (f >> 3) & 15
    // along m: a wave reads 8 rows x 128 contiguous bytes, and its scalar
    // stores to the [m][r] stage meet at most two lanes per bank)
    const int tr0 = (f0 & 7) + 8 * (f0 >> 7), tq0 = (f0 >> 3) & 15;
    const int tr1 = (f1 & 7) + 8 * (f1 >> 7), tq1 = (f1 >> 3) & 15;
    const float *pa0 = TA ? A + (int64_t)(rbeg + tr0) * M + m0 + 4 * tq0
                          : A + (int64_t)(m0 + (f0 >> 3)) * R + 4 * (f0 & 7) + rbeg;
    const float *pa1 = TA ? A + (int64_t)(rbeg + tr1) * M + m0 + 4 * tq1
                          : A + (int64_t)(m0 + (f1 >> 3)) * R + 4 * (f1 & 7) + rbeg;
    const int64_t astep = TA ? (int64_t)C1_RC * M : C1_RC;
    const float *px0 = X + c1_off(j0 + 4 * (f0 & 15), f0 >> 4, R, P) + (int64_t)rbeg * P;
    const float *px1 = X + c1_off(j0 + 4 * (f1 & 15), f1 >> 4, R, P) + (int64_t)rbeg * P;
    float *const sa0 = TA ? lds + 4 * tq0 * C1_AS + tr0 : lds + (f0 >> 3) * C1_AS + 4 * (f0 & 7);
    float *const sa1 = TA ? lds + 4 * tq1 * C1_AS + tr1 : lds + (f1 >> 3) * C1_AS + 4 * (f1 & 7);
    float *const sb0 = lds + C1_ASTAGE + (f0 >> 4) * C1_BS + 4 * (f0 & 15);
    float *const sb1 = lds + C1_ASTAGE + (f1 >> 4) * C1_BS + 4 * (f1 & 15);
    const int64_t xstep = (int64_t)C1_RC * P;
    // One chunk in flight in registers: chunk c + 1's loads are issued before
    // chunk c's MFMAs and stored to the other LDS stage after them; the load
    // past the last chunk re-reads it (no branch: a conditional load made the
    // compiler wait for every load in flight).  Macros over named registers:
    // float4 arrays captured by lambdas went to scratch, whose stores waited
    // for the loads at issue.  (Three chunks in flight measured 2-8 % slower,
    // profiles/r14/conv1x1_variants.txt.)
    float4 g0a0, g0a1, g0b0, g0b1;
#define C1_GLOAD(g, c)                                                         \
    {                                                                          \
        const int cc_ = min((c), nchunk - 1);                                  \
        g##a0 = *reinterpret_cast<const float4 *>(pa0 + astep * cc_);          \
        g##a1 = *reinterpret_cast<const float4 *>(pa1 + astep * cc_);          \
        g##b0 = *reinterpret_cast<const float4 *>(px0 + xstep * cc_);          \
        g##b1 = *reinterpret_cast<const float4 *>(px1 + xstep * cc_);          \
    }
#define C1_LSTORE(g, buf)                                                      \
    {                                                                          \
        const int o_ = (buf) * C1_STAGE;                                       \
        if constexpr (TA) {                                                    \
            sa0[o_] = g##a0.x; sa0[o_ + C1_AS] = g##a0.y;                      \
            sa0[o_ + 2 * C1_AS] = g##a0.z; sa0[o_ + 3 * C1_AS] = g##a0.w;      \
            sa1[o_] = g##a1.x; sa1[o_ + C1_AS] = g##a1.y;                      \
            sa1[o_ + 2 * C1_AS] = g##a1.z; sa1[o_ + 3 * C1_AS] = g##a1.w;      \
        } else {                                                               \
            *reinterpret_cast<float4 *>(sa0 + o_) = g##a0;                     \
            *reinterpret_cast<float4 *>(sa1 + o_) = g##a1;                     \
        }                                                                      \
        *reinterpret_cast<float4 *>(sb0 + o_) = g##b0;                         \
        *reinterpret_cast<float4 *>(sb1 + o_) = g##b1;                         \
    }

    const int mh = w >> 1, jh = w & 1, h = lane >> 5, l32 = lane & 31;
    // MFMA t (0..15) of a chunk reduces over r = t (lane half 0) and 16 + t
    // (half 1): a lane's A values are the contiguous run A[m][16 h .. 16 h +
    // 15] (four 16-byte reads; rows 144 B apart hit distinct banks), its B
    // values B[16 h + t][j] (ds_read2_b32 pairs).  All of a chunk's operand
    // reads are issued before its MFMAs (one LDS latency per chunk, the MFMAs
    // then wait on counted reads).
    const int arow = (mh * 32 + l32) * C1_AS + 16 * h;
    const int bcol = 16 * h * C1_BS + jh * 32 + l32;
    f32x16 acc = f32x16{};
#define C1_CHUNK(buf)                                                          \
    {                                                                          \
        const float *As_ = lds + (buf) * C1_STAGE;                             \
        const float *Bs_ = As_ + C1_ASTAGE;                                    \
        float4 a4_[4];                                                         \
        float bv_[16];                                                         \
        _Pragma("unroll") for (int q = 0; q < 4; ++q) a4_[q] =                 \
            *reinterpret_cast<const float4 *>(As_ + arow + 4 * q);             \
        _Pragma("unroll") for (int t = 0; t < 16; ++t) bv_[t] = Bs_[bcol + t * C1_BS]; \
        __builtin_amdgcn_sched_barrier(0);                                     \
        _Pragma("unroll") for (int q = 0; q < 4; ++q) {                        \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4_[q].x, bv_[4 * q], acc, 0, 0, 0);     \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4_[q].y, bv_[4 * q + 1], acc, 0, 0, 0); \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4_[q].z, bv_[4 * q + 2], acc, 0, 0, 0); \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4_[q].w, bv_[4 * q + 3], acc, 0, 0, 0); \
        }                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                     \
    }
    Y += (int64_t)blockIdx.y * J * M;
    C1_GLOAD(g0, 0);
    C1_LSTORE(g0, 0);
    __syncthreads();
    int c = 0;
    do {
        C1_GLOAD(g0, c + 1);
        __builtin_amdgcn_sched_barrier(0);
        C1_CHUNK(c & 1);
        if (c + 1 < nchunk) {
            C1_LSTORE(g0, (c + 1) & 1);
            __syncthreads();
        }
        ++c;
    } while (c < nchunk);
#undef C1_CHUNK
#undef C1_LSTORE
#undef C1_GLOAD
    // epilogue: lane (h, l32) holds rows (r & 3) + 8 (r >> 2) + 4 h of column
    // jh 32 + l32: per register one coalesced 128-byte row segment per half
    const int64_t j = j0 + jh * 32 + l32;
    const int64_t n = j / P, p = j - n * (int64_t)P;
    float *yc = Y + n * (int64_t)M * P + p;
    const int mr = m0 + mh * 32 + 4 * h;
    if (bias) {
        float bv[16];                           // all 16 loads in flight at once
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[r] = bias[mr + (r & 3) + 8 * (r >> 2)];
#pragma unroll
        for (int r = 0; r < 16; ++r) yc[(int64_t)(mr + (r & 3) + 8 * (r >> 2)) * P] = acc[r] + bv[r];
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) yc[(int64_t)(mr + (r & 3) + 8 * (r >> 2)) * P] = acc[r];
    }
}

// weight gradient partial of slice blockIdx.y: part[s][K][C] over columns
// [s * cps, (s + 1) * cps) of gy [N][K][P] and x [N][C][P]
__global__ __launch_bounds__(C1_T) void c1_wgrad_kernel(const float *__restrict__ gy,
                                                        const float *__restrict__ x,
                                                        float *__restrict__ part, int K, int C,
                                                        int P, int64_t J, int64_t cps,
                                                        int accum) {
    __shared__ float lds[2 * 2 * C1_WS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cb_n = C / 64;
    const int kb = blockIdx.x / cb_n, cb = blockIdx.x - kb * cb_n;
    const int s = blockIdx.y;
    const int64_t jbeg = (int64_t)s * cps;
    const int64_t jend = min(J, jbeg + cps);
    const int k0 = kb * 64, c0 = cb * 64;
    // chunk loads: 64 rows x 32 columns per operand = 512 float4, thread ->
    // (row f / 8, quad f % 8); the thread's column (n, p) of the next chunk to
    // load advances by one chunk per load ((dn, dp) = the chunk's 32 columns
    // split over images once, no division per chunk) and stays on the last
    // chunk.  One chunk in flight in registers, as c1_gemm.
    const int q4 = 4 * (tid & 7);
    int cn = (int)((jbeg + q4) / P), cp = (int)((jbeg + q4) - (int64_t)cn * P);
    const int dn = C1_RC / P, dp = C1_RC - (C1_RC / P) * P;
    const int64_t gplane = (int64_t)K * P, xplane = (int64_t)C * P;
    const int row0 = tid >> 3, row1 = (tid + C1_T) >> 3;
    const float *gy0 = gy + (int64_t)(k0 + row0) * P, *gy1 = gy + (int64_t)(k0 + row1) * P;
    const float *x0 = x + (int64_t)(c0 + row0) * P, *x1 = x + (int64_t)(c0 + row1) * P;
    float *const sa0 = lds + row0 * C1_AS + q4, *const sa1 = lds + row1 * C1_AS + q4;
    const int nchunk = (int)((jend - jbeg) / C1_RC);
    int nload = 0;                              // chunks whose loads are issued
    float4 g0a0, g0a1, g0b0, g0b1;
#define C1_GLOAD(g)                                                            \
    {                                                                          \
        const int64_t go_ = cn * gplane + cp, xo_ = cn * xplane + cp;          \
        g##a0 = *reinterpret_cast<const float4 *>(gy0 + go_);                  \
        g##a1 = *reinterpret_cast<const float4 *>(gy1 + go_);                  \
        g##b0 = *reinterpret_cast<const float4 *>(x0 + xo_);                   \
        g##b1 = *reinterpret_cast<const float4 *>(x1 + xo_);                   \
        if (++nload < nchunk) {                                                \
            cp += dp;                                                          \
            cn += dn;                                                          \
            if (cp >= P) {                                                     \
                cp -= P;                                                       \
                ++cn;                                                          \
            }                                                                  \
        }                                                                      \
    }
#define C1_LSTORE(g, buf)                                                      \
    {                                                                          \
        const int o_ = (buf) * 2 * C1_WS;                                      \
        *reinterpret_cast<float4 *>(sa0 + o_) = g##a0;                         \
        *reinterpret_cast<float4 *>(sa1 + o_) = g##a1;                         \
        *reinterpret_cast<float4 *>(sa0 + o_ + C1_WS) = g##b0;                 \
        *reinterpret_cast<float4 *>(sa1 + o_ + C1_WS) = g##b1;                 \
    }
    const int kh = w >> 1, ch = w & 1, h = lane >> 5, l32 = lane & 31;
    // MFMA t of a chunk reduces over columns t and 16 + t (lane halves): each
    // lane's operands are contiguous 16-float runs of its gy and x rows, all
    // 8 reads issued before the chunk's MFMAs
    const int arow = (kh * 32 + l32) * C1_AS + 16 * h;
    const int brow = (ch * 32 + l32) * C1_AS + 16 * h;
    f32x16 acc = f32x16{};
#define C1_CHUNK(buf)                                                          \
    {                                                                          \
        const float *As_ = lds + (buf) * 2 * C1_WS;                            \
        const float *Bs_ = As_ + C1_WS;                                        \
        float4 a4_[4], b4_[4];                                                 \
        _Pragma("unroll") for (int q = 0; q < 4; ++q) {                        \
            a4_[q] = *reinterpret_cast<const float4 *>(As_ + arow + 4 * q);    \
            b4_[q] = *reinterpret_cast<const float4 *>(Bs_ + brow + 4 * q);    \
        }                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                     \
        _Pragma("unroll") for (int q = 0; q < 4; ++q) {                        \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4_[q].x, b4_[q].x, acc, 0, 0, 0); \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4_[q].y, b4_[q].y, acc, 0, 0, 0); \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4_[q].z, b4_[q].z, acc, 0, 0, 0); \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4_[q].w, b4_[q].w, acc, 0, 0, 0); \
        }                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                     \
    }
    if (nchunk > 0) {
        C1_GLOAD(g0);
        C1_LSTORE(g0, 0);
        __syncthreads();
        int c = 0;
        do {
            C1_GLOAD(g0);
            __builtin_amdgcn_sched_barrier(0);
            C1_CHUNK(c & 1);
            if (c + 1 < nchunk) {
                C1_LSTORE(g0, (c + 1) & 1);
                __syncthreads();
            }
            ++c;
        } while (c < nchunk);
    }
#undef C1_CHUNK
#undef C1_LSTORE
#undef C1_GLOAD
    float *o = part + (int64_t)s * K * C;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int k = k0 + kh * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float *d = o + (int64_t)k * C + c0 + ch * 32 + l32;
        *d = accum ? *d + acc[r] : acc[r];      // accum: one slice straight into dW
    }
}

// ---- LDS-DMA forms (C1_DMA) --------------------------------------------------
// The register-staged kernels above keep one chunk in flight: at the deep
// layers (16-32 chunks per block, 256-512 blocks, one wave per SIMD) each
// chunk costs one global-load latency, and a build without MFMAs took 60-70 %
// of their time (profiles/r14/conv1x1_variants.txt).  These forms move the
// operands global -> LDS by global_load_lds_dwordx4 (1 KiB per wave
// instruction, no registers, no LDS store instructions) with C1_STAGES - 1
// chunks in flight.  Same tiles, same MFMA operands in the same order, so the
// results are bit-identical to the register-staged kernels.
//   [row][32] operands (the forward's A = W, both wgrad operands): 8 rows of
//   128 B per piece, the 16-byte quad Q of row m at slot Q ^ ((m >> 1) & 7)
//   (the source lane picks the quad, so the swizzle costs nothing): a lane's
//   ds_read_b128 of row m (16 lanes per cycle, rows m0 .. m0 + 15) hit 16
//   distinct 16-byte bank groups.
//   [row][64] operands (X, and A^T for the input gradient): 4 rows of 256 B per
//   piece, pieces 1056 B apart, so rows r and r + 16 (the two lane halves of
//   one ds_read_b32) sit on opposite bank halves.
#ifndef C1_DMA
#define C1_DMA 1
#endif
#ifndef C1_STAGES
#define C1_STAGES 2
#endif
#ifndef C1_G2_MAX
#define C1_G2_MAX 256         // grids up to this many blocks run two wave groups per block
#endif
constexpr int C1_PIECE = 1024;
constexpr int C1_PPAD = C1_PIECE + 32;
constexpr int C1D_OPER = 8 * C1_PPAD;          // bytes of one operand of a stage
constexpr int C1D_STAGE = 2 * C1D_OPER;

__device__ __forceinline__ int c1_swz(int row) { return (row >> 1) & 7; }

// this wave's pieces of its k newest chunks may stay in flight (4 per chunk)
__device__ __forceinline__ void c1_wait_chunks(int k) {
    if (k >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (k == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (k == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// G wave groups of 4 (G = 2: 8 waves, two per SIMD): group g takes chunks
// g, g + G, ... of the block's reduction (a step = G chunks, one per group,
// each group's waves moving its own chunk), so one group's barrier waits,
// LDS reads and DMA issue overlap the other's MFMAs; the groups' sums are
// added at the end (group 0's + group 1's, a fixed order).  G = 1 is the
// register-staged kernel's accumulation order, bit for bit.
template <bool TA, int S, int G>
__global__ __launch_bounds__(C1_T * G) void c1_gemm_dma_kernel(const float *__restrict__ A,
                                                               const float *__restrict__ X,
                                                               const float *__restrict__ bias,
                                                               float *__restrict__ Y, int M, int R,
                                                               int P, int64_t J, int cps) {
    static_assert(S >= 2 && S <= 5, "c1_wait_chunks covers up to 3 steps in flight");
    static_assert(G == 1 || G == 2, "one or two wave groups");
    extern __shared__ float4 c1_dyn[];
    const char *const lds = reinterpret_cast<const char *>(c1_dyn);
    const uint32_t lds0 = lds_addr(c1_dyn);
    constexpr int GST = G * C1D_STAGE;          // bytes of one pipeline stage
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int grp = w >> 2, wl = w & 3;
    const int wu = __builtin_amdgcn_readfirstlane(wl);
    const int gu = __builtin_amdgcn_readfirstlane(grp);
    const int mb_n = M / 64;
    const int64_t jb_n = J / 64;
    const int64_t blk = xcd_order(blockIdx.x, (int)(jb_n * mb_n));
    const int mb = (int)(blk % mb_n);
    const int64_t jb = blk / mb_n;
    const int m0 = mb * 64;
    const int64_t j0 = jb * 64;
    const int rbeg = blockIdx.y * cps * C1_RC;
    const int nchunk = min(cps, R / C1_RC - (int)blockIdx.y * cps);
    const int nstep = (nchunk + G - 1) / G;

    // wave wl of a group moves pieces 2 wl and 2 wl + 1 of each operand of
    // its group's chunk.  X piece i: rows 4 i + lane / 16 of the chunk,
    // columns j0 + 4 (lane % 16) (the row part 4 i and the chunk go into the
    // uniform base)
    uint32_t vb;
    {
        const int64_t j = j0 + 4 * (lane & 15);
        const int64_t n = j / P, p = j - n * P;
        vb = (uint32_t)(((n * R + (lane >> 4)) * P + p) * 4);
    }
    uint32_t va[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if constexpr (TA) {        // A^T [R][M]: rows 4 pi + lane / 16, m0 + 4 (lane % 16)
            va[i] = (uint32_t)(((lane >> 4) * M + m0 + 4 * (lane & 15)) * 4);
        } else {                   // A [M][R]: row 8 pi + lane / 8, swizzled quad
            const int m = 8 * (2 * wu + i) + (lane >> 3);
            const int q = (lane & 7) ^ c1_swz(m);
            va[i] = (uint32_t)(((int64_t)(m0 + m) * R + 4 * q) * 4);
        }
    }
    // step i into stage s: this group's chunk G i + g (a group past the last
    // chunk reloads it, so every wave has the same pieces in flight)
    auto issue = [&](int i, int s) {
        const int r = rbeg + C1_RC * min(G * i + gu, nchunk - 1);
        const uint32_t st = lds0 + (uint32_t)(s * GST + gu * C1D_STAGE);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int pi = 2 * wu + k;
            if constexpr (TA)
                glds16(va[k], A + (int64_t)(r + 4 * pi) * M, st + (uint32_t)(pi * C1_PPAD));
            else
                glds16(va[k], A + r, st + (uint32_t)(pi * C1_PIECE));
            glds16(vb, X + (int64_t)(r + 4 * pi) * P, st + (uint32_t)(C1D_OPER + pi * C1_PPAD));
        }
    };

    const int mh = wl >> 1, jh = wl & 1, h = lane >> 5, l32 = lane & 31;
    const int am = mh * 32 + l32;
    // byte offsets in a stage: MFMA t reduces over r = 16 h + t (as c1_gemm)
    const int boff = grp * C1D_STAGE + C1D_OPER + 4 * h * C1_PPAD + (jh * 32 + l32) * 4;
    const int aoff = grp * C1D_STAGE + (TA ? 4 * h * C1_PPAD + am * 4 : am * 128);
    f32x16 acc = f32x16{};
    Y += (int64_t)blockIdx.y * J * M;
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (s < nstep) issue(s, s);
    int sc = 0;                                 // stage of step i
    for (int i = 0; i < nstep; ++i) {
        c1_wait_chunks(min(S - 2, nstep - 1 - i));
        __syncthreads();                        // step i landed; step i - 1 read by all
        if (i + S - 1 < nstep) issue(i + S - 1, sc == 0 ? S - 1 : sc - 1);
        if (G * i + gu < nchunk) {
            const char *st = lds + sc * GST;
            float av[16], bv[16];
            if constexpr (TA) {
#pragma unroll
                for (int t = 0; t < 16; ++t)
                    av[t] = *reinterpret_cast<const float *>(st + aoff + (t >> 2) * C1_PPAD +
                                                             (t & 3) * 256);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v = *reinterpret_cast<const float4 *>(
                        st + aoff + (((4 * h + q) ^ c1_swz(am)) * 16));
                    av[4 * q] = v.x;
                    av[4 * q + 1] = v.y;
                    av[4 * q + 2] = v.z;
                    av[4 * q + 3] = v.w;
                }
            }
#pragma unroll
            for (int t = 0; t < 16; ++t)
                bv[t] = *reinterpret_cast<const float *>(st + boff + (t >> 2) * C1_PPAD +
                                                         (t & 3) * 256);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < 16; ++t)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t], bv[t], acc, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        sc = sc == S - 1 ? 0 : sc + 1;
    }
    if constexpr (G == 2) {
        // group 1's sums through LDS (the stages are free after the barrier)
        float *red = reinterpret_cast<float *>(c1_dyn) + wl * 16 * 64 + lane;
        __syncthreads();
        if (grp == 1) {
#pragma unroll
            for (int r = 0; r < 16; ++r) red[r * 64] = acc[r];
        }
        __syncthreads();
        if (grp == 1) return;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = acc[r] + red[r * 64];
    }
    // epilogue: as c1_gemm
    const int64_t j = j0 + jh * 32 + l32;
    const int64_t n = j / P, p = j - n * (int64_t)P;
    float *yc = Y + n * (int64_t)M * P + p;
    const int mr = m0 + mh * 32 + 4 * h;
    if (bias) {
        float bb[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) bb[r] = bias[mr + (r & 3) + 8 * (r >> 2)];
#pragma unroll
        for (int r = 0; r < 16; ++r) yc[(int64_t)(mr + (r & 3) + 8 * (r >> 2)) * P] = acc[r] + bb[r];
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) yc[(int64_t)(mr + (r & 3) + 8 * (r >> 2)) * P] = acc[r];
    }
}

// weight gradient: both operands [row][32 columns] (swizzled pieces); a
// chunk's 32 columns lie in one image (P % 32 == 0) or span 32 / P whole
// images (32 % P == 0), so a lane's source is a fixed offset from the
// chunk's uniform base.  G wave groups as c1_gemm_dma (G = 1: the
// register-staged kernel's order, bit for bit).
template <int S, int G>
__global__ __launch_bounds__(C1_T * G) void c1_wgrad_dma_kernel(const float *__restrict__ gy,
                                                                const float *__restrict__ x,
                                                                float *__restrict__ part, int K,
                                                                int C, int P, int64_t J,
                                                                int64_t cps, int accum) {
    static_assert(S >= 2 && S <= 5, "c1_wait_chunks covers up to 3 steps in flight");
    static_assert(G == 1 || G == 2, "one or two wave groups");
    extern __shared__ float4 c1_dyn[];
    const char *const lds = reinterpret_cast<const char *>(c1_dyn);
    const uint32_t lds0 = lds_addr(c1_dyn);
    constexpr int WST = 2 * 8 * C1_PIECE;       // chunk bytes: gy rows, then x rows
    constexpr int GST = G * WST;                // bytes of one pipeline stage
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int grp = w >> 2, wl = w & 3;
    const int wu = __builtin_amdgcn_readfirstlane(wl);
    const int gu = __builtin_amdgcn_readfirstlane(grp);
    const int cb_n = C / 64;
    const int kb = blockIdx.x / cb_n, cb = blockIdx.x - kb * cb_n;
    const int s = blockIdx.y;
    const int64_t jbeg = (int64_t)s * cps;
    const int64_t jend = min(J, jbeg + cps);
    const int k0 = kb * 64, c0 = cb * 64;
    const int nchunk = (int)((jend - jbeg) / C1_RC);
    const int nstep = (nchunk + G - 1) / G;
    // lane part of piece pi (rows 8 pi + lane / 8, quad q swizzled): column
    // 4 q of the chunk = image 4 q / P, pixel 4 q % P past the chunk's start
    uint32_t vg[2], vx[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = 8 * (2 * wu + i) + (lane >> 3);
        const int q = (lane & 7) ^ c1_swz(row);
        const int img = P >= C1_RC ? 0 : (4 * q) / P;
        const int pp = P >= C1_RC ? 4 * q : (4 * q) % P;
        vg[i] = (uint32_t)((((int64_t)img * K + row) * P + pp) * 4);
        vx[i] = (uint32_t)((((int64_t)img * C + row) * P + pp) * 4);
    }
    // step i into stage sidx: this group's chunk G i + g (past the last chunk:
    // the last chunk again, so every wave has the same pieces in flight)
    auto issue = [&](int i, int sidx) {
        const uint32_t jc = (uint32_t)(jbeg + C1_RC * min(G * i + gu, nchunk - 1));
        const uint32_t cn = jc / (uint32_t)P, cp = jc - cn * (uint32_t)P;
        const uint32_t st = lds0 + (uint32_t)(sidx * GST + gu * WST);
        const float *bg = gy + ((int64_t)cn * K + k0) * (int64_t)P + cp;
        const float *bx = x + ((int64_t)cn * C + c0) * (int64_t)P + cp;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int pi = 2 * wu + k;
            glds16(vg[k], bg, st + (uint32_t)(pi * C1_PIECE));
            glds16(vx[k], bx, st + (uint32_t)(8 * C1_PIECE + pi * C1_PIECE));
        }
    };
    const int kh = wl >> 1, ch = wl & 1, h = lane >> 5, l32 = lane & 31;
    const int ar = kh * 32 + l32, br = ch * 32 + l32;
    const int ao = grp * WST + ar * 128, bo = grp * WST + 8 * C1_PIECE + br * 128;
    f32x16 acc = f32x16{};
#pragma unroll
    for (int i = 0; i < S - 1; ++i)
        if (i < nstep) issue(i, i);
    int sc = 0;
    for (int i = 0; i < nstep; ++i) {
        c1_wait_chunks(min(S - 2, nstep - 1 - i));
        __syncthreads();
        if (i + S - 1 < nstep) issue(i + S - 1, sc == 0 ? S - 1 : sc - 1);
        if (G * i + gu < nchunk) {
            const char *st = lds + sc * GST;
            float4 a4[4], b4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a4[q] = *reinterpret_cast<const float4 *>(st + ao + (((4 * h + q) ^ c1_swz(ar)) * 16));
                b4[q] = *reinterpret_cast<const float4 *>(st + bo + (((4 * h + q) ^ c1_swz(br)) * 16));
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[q].x, b4[q].x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[q].y, b4[q].y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[q].z, b4[q].z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[q].w, b4[q].w, acc, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        sc = sc == S - 1 ? 0 : sc + 1;
    }
    if constexpr (G == 2) {
        float *red = reinterpret_cast<float *>(c1_dyn) + wl * 16 * 64 + lane;
        __syncthreads();
        if (grp == 1) {
#pragma unroll
            for (int r = 0; r < 16; ++r) red[r * 64] = acc[r];
        }
        __syncthreads();
        if (grp == 1) return;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = acc[r] + red[r * 64];
    }
    float *o = part + (int64_t)s * K * C;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int k = k0 + kh * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float *d = o + (int64_t)k * C + c0 + ch * 32 + l32;
        *d = accum ? *d + acc[r] : acc[r];
    }
}

// out[i] = sum over slabs [g G, min(S, g G + G)) of n4 float4 each for group
// g = blockIdx.y, in slab order (+ bias[(i / (rowlen / 4)) % nb] when bias):
// the first level of a two-level fixed-order slab sum (G slabs per group;
// one group: the whole sum), 8 loads in flight per thread
__global__ void c1_sum_kernel(const float4 *__restrict__ part, int S, int G, int64_t n4,
                              float4 *__restrict__ out, const float *__restrict__ bias,
                              int rowlen, int nb, int accum) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const int s0 = blockIdx.y * G, s1 = min(S, s0 + G);
    float4 a = part[(int64_t)s0 * n4 + i];
    for (int b = s0 + 1; b < s1; b += 8) {
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = (b + j < s1) ? part[(int64_t)(b + j) * n4 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (b + j < s1) {
                a.x += v[j].x; a.y += v[j].y; a.z += v[j].z; a.w += v[j].w;
            }
        }
    }
    if (bias) {
        const float bb = bias[(int)((i * 4 / rowlen) % nb)];
        a.x += bb; a.y += bb; a.z += bb; a.w += bb;
    }
    float4 *o = out + (int64_t)blockIdx.y * n4 + i;
    if (accum) {                                // a weight's later gradient contribution
        const float4 v = *o;
        a = make_float4(v.x + a.x, v.y + a.y, v.z + a.z, v.w + a.w);
    }
    *o = a;
}

constexpr int C1_GROUP = 16;
int c1_groups(int S) { return S > 2 * C1_GROUP ? (S + C1_GROUP - 1) / C1_GROUP : 0; }

// Reduction slices so that tiles x slices fills ~C1_TARGET workgroups (4 per
// CU: the kernel hides its latencies by occupancy), at least min_chunks
// chunks each: 16 for c1_gemm (a launch without the slab sum beat two slices
// + c1_sum at 16 chunks), 8 for c1_wgrad (profiles/r14/conv1x1_variants.txt)
#ifndef C1_TARGET
#define C1_TARGET 1024
#endif
#ifndef C1_MINCH_GEMM
#define C1_MINCH_GEMM 16
#endif
#ifndef C1_MINCH_WGRAD
#define C1_MINCH_WGRAD 8
#endif
int c1_slices(int tiles, int64_t nchunk, int min_chunks, int target = C1_TARGET) {
    int64_t S = (target + tiles - 1) / tiles;
    S = min(S, max((int64_t)1, nchunk / min_chunks));
    return (int)max((int64_t)1, S);
}

// the slab sum of S slabs of n floats (in order; two levels above 2 G slabs)
// into out; gbuf holds the groups (c1_groups(S) slabs)
smmd_status c1_reduce(const float *part, int S, int64_t n, float *gbuf, float *out,
                      const float *bias, int rowlen, int nb, hipStream_t st, int accum = 0) {
    const int64_t n4 = n / 4;
    const unsigned gx = (unsigned)((n4 + 255) / 256);
    const int ng = c1_groups(S);
    if (ng > 0) {
        c1_sum_kernel<<<dim3(gx, (unsigned)ng), dim3(256), 0, st>>>(
            reinterpret_cast<const float4 *>(part), S, C1_GROUP, n4,
            reinterpret_cast<float4 *>(gbuf), nullptr, 1, 1, 0);
        const smmd_status e = last_launch_status();
        if (e != SMMD_OK) return e;
        part = gbuf;
        S = ng;
    }
    c1_sum_kernel<<<dim3(gx, 1), dim3(256), 0, st>>>(reinterpret_cast<const float4 *>(part), S, S,
                                                     n4, reinterpret_cast<float4 *>(out), bias,
                                                     rowlen, nb, accum);
    return last_launch_status();
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

}  // namespace smmd

using namespace smmd;

extern "C" int smmd_conv1x1_supported(int n, int r, int m, int p) {
    // r: the reduction channels, m: the output channels, p: pixels per image
    const int64_t J = (int64_t)n * p;
    return n > 0 && r > 0 && m > 0 && p > 0 && m % 64 == 0 && r % C1_RC == 0 && p % 4 == 0 &&
           J % 64 == 0 && (int64_t)n * (r > m ? r : m) * p < (1ll << 40);
}

namespace {
int c1_gemm_slices(int n, int r, int m, int p) {
    const int64_t J = (int64_t)n * p;
    const int64_t tiles = (J / 64) * (m / 64);
    return tiles >= C1_TARGET ? 1 : c1_slices((int)tiles, r / C1_RC, C1_MINCH_GEMM);
}
}  // namespace

extern "C" size_t smmd_conv1x1_workspace_bytes(int n, int r, int m, int p) {
    if (!smmd_conv1x1_supported(n, r, m, p)) return 0;
    const int S = c1_gemm_slices(n, r, m, p);
    if (S == 1) return 0;
    return (size_t)(S + c1_groups(S)) * n * m * p * sizeof(float);
}

static smmd_status c1_gemm_launch(const float *a, const float *x, const float *bias, float *y,
                                  int n, int r, int m, int p, void *ws, size_t ws_bytes, bool ta,
                                  smmd_stream_t stream) {
    if (!a || !x || !y) return SMMD_EINVAL;
    if (!smmd_conv1x1_supported(n, r, m, p)) return SMMD_EUNSUPPORTED;
    if (!aligned16(a) || !aligned16(x) || !aligned16(y)) return SMMD_EINVAL;
    const int64_t J = (int64_t)n * p;
    const int64_t blocks = (J / 64) * (m / 64);
    if (blocks > 0x7fffffff) return SMMD_EUNSUPPORTED;
    const int S = c1_gemm_slices(n, r, m, p);
    const size_t need = smmd_conv1x1_workspace_bytes(n, r, m, p);
    if (need && (!ws || ws_bytes < need || !aligned16(ws))) return SMMD_EWORKSPACE;
    const int nch = r / C1_RC;
    const int cps = (nch + S - 1) / S;
    const int Sused = (nch + cps - 1) / cps;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    float *part = Sused > 1 ? static_cast<float *>(ws) : y;
    const dim3 grid((unsigned)blocks, (unsigned)Sused);
#if C1_DMA
    // the DMA form's lane offsets are 32-bit byte offsets
    if ((int64_t)n * r * p * 4 < (1ll << 31) && (int64_t)m * r * 4 < (1ll << 31)) {
        // two wave groups when the grid leaves a CU one block (one wave per SIMD)
        const bool g2 = blocks * Sused <= C1_G2_MAX && nch / Sused >= 2;
        static bool attr = false;
        constexpr int lds1 = C1_STAGES * C1D_STAGE, lds2 = 2 * C1_STAGES * C1D_STAGE;
        if (!attr) {
            const void *ks[4] = {reinterpret_cast<const void *>(c1_gemm_dma_kernel<true, C1_STAGES, 1>),
                                 reinterpret_cast<const void *>(c1_gemm_dma_kernel<false, C1_STAGES, 1>),
                                 reinterpret_cast<const void *>(c1_gemm_dma_kernel<true, C1_STAGES, 2>),
                                 reinterpret_cast<const void *>(c1_gemm_dma_kernel<false, C1_STAGES, 2>)};
            for (int i = 0; i < 4; ++i)
                if (hipFuncSetAttribute(ks[i], hipFuncAttributeMaxDynamicSharedMemorySize,
                                        i < 2 ? lds1 : lds2) != hipSuccess)
                    return SMMD_EHIP;
            attr = true;
        }
        const float *b1 = Sused > 1 ? nullptr : bias;
        if (g2) {
            auto kd = ta ? c1_gemm_dma_kernel<true, C1_STAGES, 2> : c1_gemm_dma_kernel<false, C1_STAGES, 2>;
            kd<<<grid, dim3(2 * C1_T), lds2, st>>>(a, x, b1, part, m, r, p, J, cps);
        } else {
            auto kd = ta ? c1_gemm_dma_kernel<true, C1_STAGES, 1> : c1_gemm_dma_kernel<false, C1_STAGES, 1>;
            kd<<<grid, dim3(C1_T), lds1, st>>>(a, x, b1, part, m, r, p, J, cps);
        }
    } else
#endif
    {
        auto k = ta ? c1_gemm_kernel<true> : c1_gemm_kernel<false>;
        k<<<grid, dim3(C1_T), 0, st>>>(a, x, Sused > 1 ? nullptr : bias, part, m, r, p, J, cps);
    }
    smmd_status e = last_launch_status();
    if (e != SMMD_OK || Sused == 1) return e;
    const int64_t total = J * m;
    return c1_reduce(part, Sused, total, part + (size_t)Sused * total, y, bias, p, m, st);
}

extern "C" smmd_status smmd_conv1x1(const float *a, const float *x, const float *bias, float *y,
                                    int n, int r, int m, int p, void *ws, size_t ws_bytes,
                                    smmd_stream_t stream) {
    return c1_gemm_launch(a, x, bias, y, n, r, m, p, ws, ws_bytes, false, stream);
}

// y [n][m][p] = a^T x (+ bias) with a [r][m]: the input gradient of a 1x1 conv
// straight from its weight W [K = r][C = m] (dx = W^T gy)
extern "C" smmd_status smmd_conv1x1_t(const float *a, const float *x, const float *bias, float *y,
                                      int n, int r, int m, int p, void *ws, size_t ws_bytes,
                                      smmd_stream_t stream) {
    return c1_gemm_launch(a, x, bias, y, n, r, m, p, ws, ws_bytes, true, stream);
}

extern "C" int smmd_conv1x1_wgrad_supported(int n, int c, int k, int p) {
    const int64_t J = (int64_t)n * p;
    return n > 0 && c > 0 && k > 0 && p > 0 && c % 64 == 0 && k % 64 == 0 && p % 4 == 0 &&
           J % C1_RC == 0 && (int64_t)n * (c > k ? c : k) * p < (1ll << 40);
}

namespace {
#ifndef C1_WG_G
#define C1_WG_G 2             // wave groups of the LDS-DMA weight gradient
#endif
// the LDS-DMA weight gradient: a chunk's 32 columns in one image or over
// whole images, 32-bit column indices
bool c1_wgrad_dma(int n, int p) {
    return C1_DMA && (p % C1_RC == 0 || C1_RC % p == 0) && (int64_t)n * p < (1ll << 31);
}
// column slices: ~C1_TARGET / G workgroups of G wave groups, >= 8 chunks per group
int c1_wgrad_slices(int n, int c, int k, int p) {
    const int g = c1_wgrad_dma(n, p) ? C1_WG_G : 1;
    return c1_slices((k / 64) * (c / 64), (int64_t)n * p / C1_RC, C1_MINCH_WGRAD * g, C1_TARGET / g);
}
}  // namespace

extern "C" size_t smmd_conv1x1_wgrad_workspace_bytes(int n, int c, int k, int p) {
    if (!smmd_conv1x1_wgrad_supported(n, c, k, p)) return 0;
    const int S = c1_wgrad_slices(n, c, k, p);
    return S > 1 ? (size_t)(S + c1_groups(S)) * k * c * sizeof(float) : 0;
}

static smmd_status c1_wgrad_launch(const float *gy, const float *x, float *gw, int n, int c,
                                   int k, int p, void *ws, size_t ws_bytes, int accum,
                                   smmd_stream_t stream) {
    if (!gy || !x || !gw) return SMMD_EINVAL;
    if (!smmd_conv1x1_wgrad_supported(n, c, k, p)) return SMMD_EUNSUPPORTED;
    if (!aligned16(gy) || !aligned16(x) || !aligned16(gw)) return SMMD_EINVAL;
    const int64_t J = (int64_t)n * p;
    const int tiles = (k / 64) * (c / 64);
    const int64_t nch = J / C1_RC;
    const int S = c1_wgrad_slices(n, c, k, p);
    const size_t need = smmd_conv1x1_wgrad_workspace_bytes(n, c, k, p);
    if (need && (!ws || ws_bytes < need || !aligned16(ws))) return SMMD_EWORKSPACE;
    // columns per slice: whole chunks
    const int64_t cps = ((nch + S - 1) / S) * C1_RC;
    const int Sused = (int)((J + cps - 1) / cps);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    float *part = Sused > 1 ? static_cast<float *>(ws) : gw;
    const dim3 grid((unsigned)tiles, (unsigned)Sused);
#if C1_DMA
    if (c1_wgrad_dma(n, p)) {
        constexpr int lds = C1_WG_G * C1_STAGES * 2 * 8 * C1_PIECE;
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute(reinterpret_cast<const void *>(c1_wgrad_dma_kernel<C1_STAGES, C1_WG_G>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
                return SMMD_EHIP;
            attr = true;
        }
        c1_wgrad_dma_kernel<C1_STAGES, C1_WG_G><<<grid, dim3(C1_WG_G * C1_T), lds, st>>>(
            gy, x, part, k, c, p, J, cps, Sused == 1 ? accum : 0);
    } else
#endif
    {
        c1_wgrad_kernel<<<grid, dim3(C1_T), 0, st>>>(gy, x, part, k, c, p, J, cps,
                                                     Sused == 1 ? accum : 0);
    }
    smmd_status e = last_launch_status();
    if (e != SMMD_OK || Sused == 1) return e;
    const int64_t total = (int64_t)k * c;
    return c1_reduce(part, Sused, total, part + (size_t)Sused * total, gw, nullptr, 1, 1, st,
                     accum);
}

extern "C" smmd_status smmd_conv1x1_wgrad(const float *gy, const float *x, float *gw, int n,
                                          int c, int k, int p, void *ws, size_t ws_bytes,
                                          smmd_stream_t stream) {
    return c1_wgrad_launch(gy, x, gw, n, c, k, p, ws, ws_bytes, 0, stream);
}

extern "C" smmd_status smmd_conv1x1_wgrad_acc(const float *gy, const float *x, float *gw, int n,
                                              int c, int k, int p, void *ws, size_t ws_bytes,
                                              smmd_stream_t stream) {
    return c1_wgrad_launch(gy, x, gw, n, c, k, p, ws, ws_bytes, 1, stream);
}
