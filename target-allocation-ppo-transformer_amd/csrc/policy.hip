// policy.hip -- K4: fused TransformerActorCritic forward (networks/transformer_net.py:15-144) on
// gfx950, fp32-accurate (the reference's dtype): every encoder GEMM as split products on the f16
// MFMA (v_mfma_f32_16x16x32_f16, each operand as two fp16 planes x1 = f16(x), x2 = f16((x - x1) 2^11),
// three MFMAs per block, fp32 accumulation), the embeddings (K = 14) and the heads on
// the f32 MFMA (v_mfma_f32_16x16x4_f32, exact fp32 products). Range of the split operands: 2^-22
// relative per product for |x| in [2^-14, 65504]; below 2^-14 an absolute floor of ~2^-36 (the
// backward therefore carries its gradients pre-scaled, BwdIO::gscale); from 65520 up the planes are
// inf / -inf and every output that reads them is non-finite (common.hpp f16_lo; the ReLUs keep NaN,
// relu_nan), never a finite wrong value.
// (The notes below on tiles and layout date from the all-f32 design and still describe the f32
// building blocks.)
//
// Work decomposition (MI355X-first):
//  * one workgroup = 4 waves = 16 samples = 80 tokens, token index tok = s * 16 + p (s = window
//    position, p = sample): every 16-column MFMA tile is one window position of the 16 samples,
//    so the last position (the only one the heads read, transformer_net.py:106,114) is exactly
//    column tile 4. B = 4096 -> 256 workgroups = one per CU.
//  * GEMMs are computed transposed, Y^T = W . X^T: the weight rows (Linear's [out][in] layout,
//    contiguous in k) are the A operand, streamed from L2 as float4 (4 k per lane = 4 MFMAs);
//    activations live in LDS as [tok][feature] rows and are the B operand, read as float4; the
//    accumulator (feature rows x token columns) is stored back as one float4 per lane.
//    Both operands use the same k permutation (k = 16*i + 4*(lane>>4) + j for MFMA j), so the
//    sum is over every k exactly once.
//  * the four waves split the output features of every GEMM; attention (5 x 5 per sample and
//    head, far too small for MFMA), LayerNorm and the 128->64->{2,1} heads run on the VALU.
//  * last-layer pruning: in the final encoder layer of each trunk only K and V are formed for
//    all 80 tokens; Q, attention, out-projection, LayerNorms and the FFN run for column tile 4
//    only (2.45 instead of 4.04 MFLOP per sample; numerically identical outputs).
//  * sampling: a = (u < p0) ? 0 : 1 with u ~ Philox(seed, offset + b) (not torch's RNG stream;
//    parity is defined on logits / logp / value / entropy for given actions).
#include "common.hpp"
#include "env_device.hpp"
#if defined(UAVHIP_POLICY_TRACE) && defined(UAVHIP_STEPS_TU) && defined(UAVHIP_ENV_FINE)
// make TRACE=1 ENVFINE=1 (k_rollout_steps only): stamps inside the grouped env step (env_group.hpp
// GTR, slots 40-47) in the same buffer as PTR, waves 0 and 4 of the first 256 workgroups
namespace uavhip { namespace pol { __device__ unsigned long long g_strace[256 * 2 * 64]; } }
#define UAVHIP_STRACE_DEFINED 1
#define GTR(id)                                                                                  \
    do {                                                                                         \
        if ((tid_x() & 255) == 0 && blockIdx.x < 256)                                        \
            ::uavhip::pol::g_strace[(blockIdx.x * 2 + (tid_x() >> 8)) * 64 + (id)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#endif
#include "env_group.hpp"
#include "policy_layout.hpp"
#include "policy_train.hpp"
// The policy code is contracted (a * b + c as one fma, v_pk_fma_f32 on float pairs): the env headers
// above switch contraction off for the rest of the translation unit at file scope (their fp64 code must
// follow the reference's operation order), which until round 6 silently applied to every function
// below too. Their templates keep the state they were parsed with; the operand-range functions that
// producer and consumer must evaluate identically keep their own contract(off). Same-box A/B
// (profiles/r06u_ab_contract.txt): k_rollout_steps 49.4 -> 48.2 us per step, the training forward
// 87.6 -> 84.5 us; every -m gpu test unchanged in outcome. EXP=91 (A/B build): uncontracted as before.
#if UAVHIP_EXP != 91
#pragma clang fp contract(fast)
#endif

namespace uavhip {
namespace pol {

constexpr int SPW = 16;         // samples per workgroup
constexpr int TOK = S * SPW;    // 80
constexpr int NW = 8;            // waves per workgroup: two per SIMD
constexpr int NTHR = NW * 64;
constexpr int LDH = D + 8;      // 136: row stride = 2 mod 16 slots of 16 B -> the MFMA operand
                                // reads/writes (lane = row i + 16 * k-group g) hit 16 distinct slots
constexpr int LDB = 3 * 64 + 8; // 200: [Q 64 | K 64 | V 64] for a chunk of 4 heads
constexpr int LDF = D + 8;
constexpr int LDX = 16;         // input rows padded 14 -> 16 (one MFMA k-block)
constexpr int LDZ = HID + 8;

typedef float f32x4 __attribute__((ext_vector_type(4)));
#ifdef UAVHIP_EXP_NOSTORE
constexpr bool kExpNoStore = true;
#else
constexpr bool kExpNoStore = false;
#endif
// make NOENV=1 (profiling builds only, wrong results): the fused rollout kernels skip the env step
// but still write the next windows -- the input windows shifted by one row, every row's constant
// feature (index 13, 1.0 in every real observation row) set -- so no position of the next step's
// windows is padding and the policy's data-dependent ring loads (a padded position reads one hot
// dummy row, ring_load) stay those of a real rollout. bench.py prices the env step as the product
// build's time minus this build's; scripts/profile_env_share.sh the same for PMC bytes. (Until round
// 4 the NOENV build left the next windows all zero -- every position but the last padded -- which also
// dropped ~41 MB per step of ring-row reads: that differential was not the env step's cost.)
#ifdef UAVHIP_EXP_NOENV
constexpr bool kExpNoEnv = true;
#else
constexpr bool kExpNoEnv = false;
#endif
// Timing build EXP=32 (profiling only, WRONG results): every ring-row load reads one hot row (the
// load still issued, its value used): the cost of the ring rows' L2 misses, by difference.
// EXP=61 / 62 / 63 (WRONG results out of range): the static operand scales / layer 0's dynamic ones
// / both compiled as 1 -- the cost of the range scaling, by difference (DESIGN.md 4a "Range").
#ifndef UAVHIP_EXP
#define UAVHIP_EXP 0
#endif
constexpr bool kExpHotRing = UAVHIP_EXP == 32;
constexpr bool kEarlyDraw = UAVHIP_EXP != 105;  // policy_block: the sampling draws at the step's start
// EXP=71 (timing only, WRONG results): the split-product GEMMs load only the blocks their callers
// prefetched (blocks >= D_ of a tile repeat them): the cost of the in-loop weight loads' latency --
// the ceiling of a deeper weight prefetch (an LDS-DMA ring). EXP=73: also every prefetch reads one
// hot 1 KiB block (the weight stream from L2 compiled out of the split GEMMs).
constexpr bool kExpNoWeightLoads = UAVHIP_EXP == 71 || UAVHIP_EXP == 73;
// The training forward's activation stores (the rows K6 and the weight-gradient GEMM read back after
// the whole forward: Q | K | V, x-hat, the embeddings, FFN hidden units, attention outputs) are
// non-temporal: they stream past the L2 instead of evicting the weights and re-read rows there.
// Same-box A/B (profiles/r06m_train_ab_nt_stores.txt): K6 104.4-108.5 -> 101.1-101.3 us at minibatch
// 4096, the forward unchanged. Not in the position-split kernels (K7, minibatch <= 256), whose next
// launch reads the rows back from the L2 (nt there: B1 / B2 +1 us each): nt = false. EXP=85 (A/B
// build): plain stores everywhere.
constexpr bool kNtAct = UAVHIP_EXP != 85;
__device__ __forceinline__ void act_st(float* p, f32x4 v, bool nt = true) {
    if (kNtAct && nt) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
    else *reinterpret_cast<f32x4*>(p) = v;
}
// EXP=84 (A/B build): K6's gradient rows for the weight-gradient GEMM (df, dz1, du, dq | dk | dv)
// as non-temporal stores too
constexpr bool kNtDy = UAVHIP_EXP == 84;
__device__ __forceinline__ void dy_st4(float* p, f32x4 v) {
    if constexpr (kNtDy) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
    else *reinterpret_cast<f32x4*>(p) = v;
}
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void dy_st2(float* p, f32x2_t v) {
    if constexpr (kNtDy) __builtin_nontemporal_store(v, reinterpret_cast<f32x2_t*>(p));
    else *reinterpret_cast<f32x2_t*>(p) = v;
}

// Phase tracing (make TRACE=1 only): waves 0 and 4 of the first 256 workgroups stamp s_memtime at
// the phase boundaries below; uavhip_policy_trace copies the stamps out. Off in the product build.
#if defined(UAVHIP_POLICY_TRACE)
#ifdef UAVHIP_STEPS_TU  // k_rollout_steps: its own buffer (the last step's stamps), uavhip_steps_trace
#define g_ptrace g_strace
#define g_btrace g_sbtrace
#endif
constexpr int kTraceSlots = 64;
#ifndef UAVHIP_STRACE_DEFINED
__device__ unsigned long long g_ptrace[256 * 2 * kTraceSlots];
#endif
#ifdef UAVHIP_TRACE_ALLWAVES  // make TRACE=1 TRACE_WAVES=8: all 8 waves of the first 64 workgroups
#define PTR(id)                                                                                  \
    do {                                                                                         \
        if ((tid_x() & 63) == 0 && blockIdx.x < 64)                                          \
            g_ptrace[(blockIdx.x * 8 + (tid_x() >> 6)) * kTraceSlots + (id)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define PTR(id)                                                                                  \
    do {                                                                                         \
        if ((tid_x() & 255) == 0 && blockIdx.x < 256)                                        \
            g_ptrace[(blockIdx.x * 2 + (tid_x() >> 8)) * kTraceSlots + (id)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#endif
__device__ unsigned long long g_btrace[256 * 2 * kTraceSlots];
#define BTR(id)                                                                                  \
    do {                                                                                         \
        if ((tid_x() & 255) == 0 && blockIdx.x < 256)                                        \
            g_btrace[(blockIdx.x * 2 + (tid_x() >> 8)) * kTraceSlots + (id)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define PTR(id) do {} while (0)
#define BTR(id) do {} while (0)
#endif

constexpr int kScr = NW * 3 * 64;  // backward scratch: per-wave in_proj bias partial rows
struct Smem {
    union {
        float x[TOK * LDX];     // input windows [tok = s*16 + p][k], k < 14 valid
        float scr[kScr];        // backward: scratch while the windows are not needed
    };
    float h[TOK * LDH];         // residual stream [tok][128]
    float big[TOK * LDB];       // QKV chunk / out-proj result / FFN hidden chunk
    float ctx[TOK * LDH];       // attention output / FFN output
    union {
        float z[SPW * LDZ];     // head hidden
        float2 red[NW * TOK];   // LayerNorm partials (mean, M2) per wave and token
    };
    float logits[SPW * 2];
    float value[SPW];
    int mask[SPW * S];          // key padding mask (transformer_net.py:52-54)
    float tmax[TOK];            // max_k |x_k| of each token's window row (layer 0's operand range)
    signed char es[2][TOK];     // per trunk and token: layer 0's input scale exponent s (from tmax)
    float a0f[4];               // per trunk: (2^-s, 2^s) of the workgroup's layer-0 attention output
    float rtab[28];             // the range table's static part (load_rtab, once per launch)
    float u01[SPW];             // the sampling draws, formed at the step's start (policy_block)
};
// Smem::rtab: the static operands' (2^-s, 2^s) pairs, then (14 max|W_e|, max|b_e| + max|pos|) and
// (D max|W_in|, max|b_in|) of layer 0 per trunk (policy_layout.hpp kRgOp / kRgE / kRgA0)
static_assert(kRtN <= 28 && kRgE + 4 == kRgA0, "Smem::rtab");

// Lane index plumbing. In the multi-step rollout TU (rollout_steps.hip) every forward helper takes
// the thread index as a leading parameter, laundered once per step by k_rollout_steps: the
// compiler then cannot hoist the body's lane-index arithmetic out of the step loop (where it would
// be spilled) and still shares it across the whole step. Elsewhere the macros are empty and the
// helpers read threadIdx.x as before.
#ifdef UAVHIP_STEPS_TU
#define TID_F unsigned tid_,
#define TID_C tid_,
#define TID_K (unsigned)threadIdx.x,
#define TIDX() tid_
#else
#define TID_F
#define TID_C
#define TID_K
#define TIDX() tid_x()
#endif
#define LANE() ((int)(TIDX() & (kWave - 1)))

// ------------------------------------------------------------------ GEMM building blocks
constexpr int KB = 128 / 16;

// The first D k-blocks of a single 16-row weight tile, loaded ahead of time (typically before the
// __syncthreads that precedes the GEMM: the barrier only drains LDS traffic, lgkmcnt(0), so these
// global loads stay in flight across it and their latency hides under the preceding phase).
template <int D>
struct APre {
    f32x4 a[D];
};
// GEMM weights are stored in MFMA fragment order (see kTileK): the A operand of 16-row tile
// `row / 16`, k-block kb is 1 KiB contiguous, lane l's float4 at 4 l. One wave instruction then
// reads 1 KiB of consecutive lines instead of 16 half-lines of 16 rows (3.3x the per-CU L2 rate
// measured on MI355X: scripts/micro/l2bw.hip).
__device__ __forceinline__ const float* frag_ptr(TID_F const float* W, int ldw, int row, int kw0) {
    return W + ((size_t)(row >> 4) * (ldw >> 4) + (kw0 >> 4)) * 256 + 4 * LANE();
}
template <int D>
__device__ __forceinline__ APre<D> prefetch(TID_F const float* __restrict__ W, int ldw, int row, int kw0) {
    const float* wp = frag_ptr(TID_C W, ldw, row, kw0);
    APre<D> r;
#pragma unroll
    for (int p = 0; p < D; ++p) r.a[p] = *reinterpret_cast<const f32x4*>(wp + 256 * p);
    return r;
}

// acc[ct] += W[row + i][kw0 + k] * X[xtok0 + 16 ct + j][k]  over k in [0, 128), one 16-row tile.
// Fully unrolled over the 8 k-blocks of 16; the loads of block i + D (weights from L2 as float4,
// activations from LDS as float4) are issued before the MFMAs of block i; blocks < D come from
// `pre`. Both operands use the same k permutation (k = 16 i + 4 (lane >> 4) + j for MFMA j).
template <int CT, int D, int NKB = KB>
__device__ __forceinline__ void gemm_tile(TID_F f32x4 (&acc)[CT], const APre<D>& pre, const float* __restrict__ W, int ldw,
                                          int row, int kw0, const float* X, int ldx, int xtok0) {
    const int l = LANE(), i16 = l & 15, g = l >> 4;
    const float* wp = frag_ptr(TID_C W, ldw, row, kw0);
    const float* xp[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) xp[ct] = X + (xtok0 + 16 * ct + i16) * ldx + 4 * g;
    f32x4 a[NKB], b[NKB][CT];
#pragma unroll
    for (int p = 0; p < D; ++p) {
        a[p] = pre.a[p];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) b[p][ct] = *reinterpret_cast<const f32x4*>(xp[ct] + 16 * p);
    }
#pragma unroll
    for (int i = 0; i < NKB; ++i) {
        if (i + D < NKB) {
            a[i + D] = *reinterpret_cast<const f32x4*>(wp + 256 * (i + D));
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) b[i + D][ct] = *reinterpret_cast<const f32x4*>(xp[ct] + 16 * (i + D));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][j], b[i][ct][j], acc[ct], 0, 0, 0);
        // keep the scheduler from hoisting every later block's loads (register pressure at 2
        // waves / SIMD): at most D blocks of operands are in flight
        __builtin_amdgcn_sched_barrier(0);
    }
}
template <int CT> constexpr int depth() { return CT == 1 ? 4 : 2; }

// The same GEMM over the 7 k-blocks kb0, kb0 + 1, ... (mod 8) -- every block but kb0 - 1, which
// the caller accumulated from registers (the wave's own LayerNorm output features, layer_tail).
template <int D>
__device__ __forceinline__ APre<D> prefetch_rot(TID_F const float* __restrict__ W, int ldw, int row, int kb0) {
    const float* wp = frag_ptr(TID_C W, ldw, row, 0);
    APre<D> r;
#pragma unroll
    for (int p = 0; p < D; ++p) r.a[p] = *reinterpret_cast<const f32x4*>(wp + 256 * ((kb0 + p) & (KB - 1)));
    return r;
}
template <int CT, int D>
__device__ __forceinline__ void gemm_tile_rot(TID_F f32x4 (&acc)[CT], const APre<D>& pre, const float* __restrict__ W,
                                              int ldw, int row, const float* X, int ldx, int xtok0, int kb0) {
    constexpr int NKB = KB - 1;
    const int l = LANE(), i16 = l & 15, g = l >> 4;
    const float* wp = frag_ptr(TID_C W, ldw, row, 0);
    const float* xp[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) xp[ct] = X + (xtok0 + 16 * ct + i16) * ldx + 4 * g;
    f32x4 a[NKB], b[NKB][CT];
#pragma unroll
    for (int p = 0; p < D; ++p) {
        const int kb = (kb0 + p) & (KB - 1);
        a[p] = pre.a[p];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) b[p][ct] = *reinterpret_cast<const f32x4*>(xp[ct] + 16 * kb);
    }
#pragma unroll
    for (int i = 0; i < NKB; ++i) {
        if (i + D < NKB) {
            const int kb = (kb0 + i + D) & (KB - 1);
            a[i + D] = *reinterpret_cast<const f32x4*>(wp + 256 * kb);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) b[i + D][ct] = *reinterpret_cast<const f32x4*>(xp[ct] + 16 * kb);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][j], b[i][ct][j], acc[ct], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int CT>
__device__ __forceinline__ void zero(f32x4 (&acc)[CT]) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// ------------------------------------------------------------------ split products on the f16 cores
// fp32-accurate GEMMs on v_mfma_f32_16x16x32_f16 (16 cycles per 16 x 16 x 32 block against 8 x 32
// for the f32 MFMA): both operands carried as two fp16 planes, x1 = f16(x), x2 = f16((x - x1) 2^11)
// (x1 + 2^-11 x2 = x to 2^-22 relative, the 2^11 keeps x2 out of the fp16 subnormals), and
//   W X^T = hi + 2^-11 lo,   hi += W1 X1,   lo += W1 X2 + W2 X1       (3 MFMAs per block)
// -- the dropped W2 X2 is 2^-22 of a product; the fp32 accumulation dominates the error
// (scripts/micro/split_gemm.hip: max error 0.42x the f32 MFMA's on the FFN1 shape, 3.6x faster).
// Weights: the packed buffer's split copies (policy_layout.hpp kSplitParam / kSplitOffs), blocks of
// 16 rows x 32 k = 1 KiB of w1 then 1 KiB of w2, lane l = r%16 + 16 ((k%32)/8) holding k%8.
// Activations: both planes of a token in one LDS row, [tok][plane 1: 128 halves | plane 2: 128 |
// pad 16] (plane 2 at + kPlane); lane (i16, g) reads 8 halves of token i16 per plane with one
// ds_read_b128. The 544-B rows put token i16 at bank offset 8 i16 (mod 64), conflict-free for
// ds_read_b128's lane groups (MI355X_MICROARCH.md LDS table) like the fp32 [tok][136] rows.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
constexpr int LDP = 2 * D + 16;      // halves per token row (both planes + pad)
constexpr int kPlane = D;            // plane 2 within the row
static_assert(TOK * LDP * 2 == TOK * LDH * 4 && kPlane + D <= LDP, "the two planes of an activation replace its fp32 copy");
// Offset of (token, column) in a plane image: the 16-B chunk index XOR-swizzled by bit 2 of the token,
// so the epilogues' ds_write_b64 (16 consecutive tokens per lane group) are at most 2-way conflicted
// (4-way without it) while the GEMMs' ds_read_b128 stay conflict-free
__device__ __forceinline__ int psw(int tok, int col) { return tok * LDP + (col ^ (((tok >> 2) & 1) << 3)); }
constexpr float kLoScale = 1.0f / 2048.0f;
// The LayerNorm's 1/sqrt(var + eps) and the attention's 1/sum(exp) on the hardware estimates
// (v_rsq_f32 / v_rcp_f32, about 1 ulp) instead of the correctly rounded sqrt + division sequences
// (~10 VALU each, on the LayerNorm and attention phases' dependency chains): same-box A/B
// (profiles/r06x_ab_rsq_rcp.txt) k_rollout_steps 48.6 -> 47.8 us per step, K6 101.8 -> 98.8 us, the
// training forward 85.8 -> 82.5 us; every -m gpu parity bar unchanged and green. EXP=94: the correctly
// rounded forms (A/B build).
__device__ __forceinline__ float ln_rstd(float v) {
    if constexpr (UAVHIP_EXP != 94) return __builtin_amdgcn_rsqf(v);
    else return 1.0f / sqrtf(v);
}
__device__ __forceinline__ float att_recip(float v) {
    if constexpr (UAVHIP_EXP != 94) return __builtin_amdgcn_rcpf(v);
    else return 1.0f / v;
}
// The forward attention's score of a query against a key over a lane's 4 head dims: one packed
// multiply and one packed FMA (3 issue slots; left to itself the compiler formed 2 packed multiplies
// and 3 adds). The 1/sqrt(16) of the scores is folded into the query (a power of two: exact).
// EXP=99 (A/B build): the previous form, the scale applied to each score.
constexpr bool kAttPk = UAVHIP_EXP != 99;
__device__ __forceinline__ float att_dot(const f32x4 q, const f32x4 k) {
    if constexpr (kAttPk) {
        f32x2_t t = f32x2_t{q.x, q.y} * f32x2_t{k.x, k.y};
        t = __builtin_elementwise_fma(f32x2_t{q.z, q.w}, f32x2_t{k.z, k.w}, t);
        return t.x + t.y;
    } else {
        return q.x * k.x + q.y * k.y + q.z * k.z + q.w * k.w;
    }
}
constexpr float kAttQ = kAttPk ? 0.25f : 1.f, kAttS = kAttPk ? 1.f : 0.25f;  // 1/sqrt(16) on q / on the score
// o += sum_j (e_j / den) v_j as (sum_j e_j v_j) / den: one scale of the sum instead of one per key
// (EXP=101 or 99: the per-key form). Not exp2(s log2e - mx log2e) as one FMA per score: for logits
// of 1e10 (windows at 1e5) the FMA's residual at the maximum itself is hundreds, exp2 of it inf or 0
// (NaN outputs in test_fused_forward_out_of_fp16_range_matches_torch); s - mx is exact there.
constexpr bool kAttMix = kAttPk && UAVHIP_EXP != 101;
template <int N>
__device__ __forceinline__ void att_mix(f32x4& o, const float (&e)[N], float inv, const f32x4 (&v)[N]) {
    if constexpr (kAttMix) {
        f32x4 a = e[0] * v[0];
#pragma unroll
        for (int j = 1; j < N; ++j) a += e[j] * v[j];
        o += a * inv;
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) o += (e[j] * inv) * v[j];
    }
}

template <int D_>
struct HPre {
    f16x8 a1[D_], a2[D_];
};
__device__ __forceinline__ const f16x8* hfrag_ptr(TID_F const float* P, int soff, int K, int row, int kw0) {
    if constexpr (UAVHIP_EXP == 73) return reinterpret_cast<const f16x8*>(P + soff) + LANE();  // timing only
    return reinterpret_cast<const f16x8*>(P + soff) + ((size_t)(row >> 4) * (K >> 5) + (kw0 >> 5)) * 128 + LANE();
}
template <int D_>
__device__ __forceinline__ HPre<D_> hprefetch(TID_F const float* __restrict__ P, int soff, int K, int row, int kw0) {
    const f16x8* wp = hfrag_ptr(TID_C P, soff, K, row, kw0);
    HPre<D_> r;
#pragma unroll
    for (int p = 0; p < D_; ++p) {
        r.a1[p] = wp[128 * p];
        r.a2[p] = wp[128 * p + 64];
    }
    return r;
}
// hi / lo[ct] += W[row + i][kw0 + k] * X[xtok0 + 16 ct + j][k] over k in [0, 128) (4 blocks of 32):
// A blocks >= D_ loaded one block ahead of their use, B (LDS) one block ahead.
// NKB blocks of 32 k; the activation planes have rows of LDX_ halves, plane 2 at + PLX halves.
// NEXT: the blocks of the NEXT tile's prefetch (nxt, from nwp) are loaded in the last D_ iterations,
// into the registers the current tile's first blocks free there -- the next GEMM's first weight
// blocks then land under this GEMM's last MFMAs instead of after them (same register peak).
template <int CT, int D_, int NKB = D / 32, int LDX_ = LDP, int PLX = kPlane, bool NEXT = false>
__device__ __forceinline__ void hgemm_tile(TID_F f32x4 (&hi)[CT], f32x4 (&lo)[CT], const HPre<D_>& pre,
                                           const float* __restrict__ P, int soff, int K, int row, int kw0,
                                           const _Float16* X, int xtok0, HPre<D_>* nxt = nullptr,
                                           const f16x8* nwp = nullptr) {
    constexpr int kPlane = PLX;
    const int l = LANE(), i16 = l & 15, g = l >> 4;
    const f16x8* wp = hfrag_ptr(TID_C P, soff, K, row, kw0);
    const _Float16* xp[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)  // the LDP images: psw's swizzle (xtok0 is a multiple of 16)
        xp[ct] = X + (xtok0 + 16 * ct + i16) * LDX_ + (LDX_ == LDP ? 8 * (g ^ ((i16 >> 2) & 1)) : 8 * g);
    f16x8 a1[NKB], a2[NKB], b1[2][CT], b2[2][CT];
#pragma unroll
    for (int p = 0; p < D_; ++p) {
        a1[p] = pre.a1[p];
        a2[p] = pre.a2[p];
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        b1[0][ct] = *reinterpret_cast<const f16x8*>(xp[ct]);
        b2[0][ct] = *reinterpret_cast<const f16x8*>(xp[ct] + kPlane);
    }
#pragma unroll
    for (int i = 0; i < NKB; ++i) {
        const int cur = i & 1;
        if (i + D_ < NKB) {
            if constexpr (kExpNoWeightLoads || (UAVHIP_EXP == 712 && CT == S) || (UAVHIP_EXP == 713 && CT == 1)) {
                // timing builds only: blocks >= D_ repeat the prefetched ones
                a1[i + D_] = a1[(i + D_) % D_];
                a2[i + D_] = a2[(i + D_) % D_];
            } else {
                a1[i + D_] = wp[128 * (i + D_)];
                a2[i + D_] = wp[128 * (i + D_) + 64];
            }
        }
        if constexpr (NEXT) {
            if (i + D_ >= NKB) {
                const int p = i - (NKB - D_);
                nxt->a1[p] = nwp[128 * p];
                nxt->a2[p] = nwp[128 * p + 64];
            }
        }
        if (i + 1 < NKB) {
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                b1[cur ^ 1][ct] = *reinterpret_cast<const f16x8*>(xp[ct] + 32 * (i + 1));
                b2[cur ^ 1][ct] = *reinterpret_cast<const f16x8*>(xp[ct] + 32 * (i + 1) + kPlane);
            }
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            hi[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], b1[cur][ct], hi[ct], 0, 0, 0);
            lo[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], b2[cur][ct], lo[ct], 0, 0, 0);
            lo[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[i], b1[cur][ct], lo[ct], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}
// ReLU that keeps NaN: the NaN a split operand beyond fp16's range produces (common.hpp f16_lo) must
// reach the outputs, and fmaxf(NaN, 0) = 0 (IEEE maxNum) swallowed it at the FFN and head ReLUs
// (measured: a 1.4e5 FFN activation gave finite, wrong values); same cost on the same box (r04f A/B)
__device__ __forceinline__ float relu_nan(float v) { return v < 0.f ? 0.f : v; }
// v -> its two planes at Y + psw(tok, c) (plane 2 at + kPlane): one 8-byte store per plane
// (common.hpp f16_split4: packed conversions. EXP=97: the per-element form, A/B build)
__device__ __forceinline__ void hsplit_store(_Float16* Y, int o, const f32x4 v) {
    f16x4 v1, v2;
    if constexpr (UAVHIP_EXP == 97) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v1[j] = (_Float16)v[j];
            v2[j] = f16_lo(v[j], v1[j]);
        }
    } else {
        f16_split4(v, v1, v2);
    }
    *reinterpret_cast<f16x4*>(Y + o) = v1;
    *reinterpret_cast<f16x4*>(Y + o + kPlane) = v2;
}
// ------------------------------------------------------------------ operand ranges of the split products
// Every activation operand is split as x 2^-s and the consuming GEMM's output multiplied by 2^s
// (policy_layout.hpp range table: s = 0 on realistic weights). Static operands (LayerNorm outputs,
// FFN hidden units, the attention output of a layer >= 1) take (2^-s, 2^s) from the table; layer 0's
// input takes s per token from the token's window-row max (Smem::tmax) and layer 0's attention
// output one s per workgroup, from the max over its 16 samples' rows (Smem::a0f). Producer and
// consumer read the same s (one evaluation, kept in LDS), so both sides always agree on it.
struct OpSc {
    float sc, inv;  // 2^-s (the producer's factor), 2^s (the consumer's)
};
__device__ __forceinline__ OpSc pow2_sc(int s) { return OpSc{ldexpf(1.0f, -s), ldexpf(1.0f, s)}; }
// The scales the kernels derive from the packed table's maxima (policy_layout.hpp range_entry) ->
// Smem::rtab, once per launch before the first barrier: every later use is an LDS read, not a scalar
// load whose lgkmcnt wait would also drain the phase's LDS traffic. Waves 0-3 take 6 entries each,
// every index a compile-time constant (the maxima they need are uniform scalar loads, one round; a
// thread per entry ran every entry's branch one after another, +1 us per kernel).
template <int W>
__device__ __forceinline__ void rtab_part(TID_F Smem& sm, const float* __restrict__ M) {
#pragma unroll
    for (int j = 0; j < kRtN / 4; ++j) {
        const int i = (kRtN / 4) * W + j;
        const float v = range_entry(M, i < kRtE ? kRgOp + i : kRgE + (i - kRtE));
        if ((TIDX() & 63) == 0) sm.rtab[i] = v;
    }
}
__device__ __forceinline__ void load_rtab(TID_F Smem& sm, const float* __restrict__ P) {
    static_assert(kRtN % 4 == 0, "4 waves");
    switch (TIDX() >> 6) {  // wave-uniform
        case 0: rtab_part<0>(TID_C sm, P + kRangeOff); break;
        case 1: rtab_part<1>(TID_C sm, P + kRangeOff); break;
        case 2: rtab_part<2>(TID_C sm, P + kRangeOff); break;
        case 3: rtab_part<3>(TID_C sm, P + kRangeOff); break;
        default: break;
    }
}
// The derived table as an earlier kernel of the same step exported it (TrainIO::rtab_out: the K7
// chain's F1 derives it once per optimizer step): one plain load per entry
// instead of the maxima's scalar loads and every entry's derivation.
__device__ __forceinline__ void load_rtab_ready(TID_F Smem& sm, const float* __restrict__ rt) {
    if (TIDX() < kRtN) sm.rtab[TIDX()] = rt[TIDX()];
}
// a uniform LDS value into an SGPR (the factors are the same in every lane: no VGPR held)
__device__ __forceinline__ float rt_uniform(const Smem& sm, int i) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sm.rtab[i])));
}
template <int trunk, int layer, int kind>
__device__ __forceinline__ OpSc op_sc(const Smem& sm) {
    constexpr int op = range_op(trunk, layer, kind);
    static_assert(op >= 0, "a static operand");
    if constexpr (UAVHIP_EXP == 61 || UAVHIP_EXP == 63) return OpSc{1.f, 1.f};  // timing builds only
    return OpSc{rt_uniform(sm, kRtOp + 2 * op), rt_uniform(sm, kRtOp + 2 * op + 1)};
}
// layer 0's input (e or e + pos) at a token whose window row has max |x_k| = m, from the trunk's
// constants ea = 14 max|W_e|, ec = max|b_e| + max|pos|; its attention output of a sample whose rows
// have max m, with a = D max|W_in|, c = max|b_in|
// (uncontracted: every site evaluates the same roundings, so a producer and its consumer agree on s)
__device__ __forceinline__ float e_bound_v(float ea, float ec, float m) {
#pragma clang fp contract(off)
    return ea * m + ec;
}
__device__ __forceinline__ OpSc e_sc_v(float ea, float ec, float m) { return pow2_sc(range_exp(e_bound_v(ea, ec, m))); }
__device__ __forceinline__ OpSc a0_sc_v(float ea, float ec, float a, float c, float m) {
#pragma clang fp contract(off)
    return pow2_sc(range_exp(a * e_bound_v(ea, ec, m) + c));
}
template <int trunk>
__device__ __forceinline__ OpSc e_sc(const Smem& sm, float m) {
    constexpr int ti = trunk_index(trunk);
    if constexpr (UAVHIP_EXP == 62 || UAVHIP_EXP == 63) return OpSc{1.f, 1.f};  // timing builds only
    return e_sc_v(rt_uniform(sm, kRtE + 2 * ti), rt_uniform(sm, kRtE + 2 * ti + 1), m);
}
// layer 0's input scale at token tok from Smem::es (gather_windows: e_sc's exponent, evaluated once
// per token): dir -1 the producer's 2^-s, +1 the consumer's 2^s
template <int trunk, int dir>
__device__ __forceinline__ float es_factor(const Smem& sm, int tok) {
    if constexpr (UAVHIP_EXP == 62 || UAVHIP_EXP == 63) return 1.f;  // timing builds only
    return ldexpf(1.0f, dir * (int)sm.es[trunk_index(trunk)][tok]);
}
// The scale of an attention output (layer 0: Smem::a0f, one per workgroup -- a uniform value, held
// in SGPRs: a per-sample factor in a VGPR across the out-projection cost the rollout loop 4 VGPR
// spills; else the static one). p: the sample (unused).
template <int trunk, int layer>
__device__ __forceinline__ OpSc att_sc(const Smem& sm, int) {
    if constexpr (layer == 0) {
        constexpr int ti = trunk_index(trunk);
        if constexpr (UAVHIP_EXP == 62 || UAVHIP_EXP == 63) return OpSc{1.f, 1.f};  // timing builds only
        return OpSc{__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sm.a0f[2 * ti]))),
                    __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sm.a0f[2 * ti + 1])))};
    } else {
        return op_sc<trunk, layer, kOpAtt>(sm);
    }
}

// Y planes [ytok0 + 16 ct + j][ycol + i] = epi(hi + 2^-11 lo + bias[row + i])
// (the operand's scale undone: x inv; the output's planes scaled: x osc)
template <int CT, bool RELU>
__device__ __forceinline__ void hstore_tile(TID_F const f32x4 (&hi)[CT], const f32x4 (&lo)[CT], const f32x4 bb,
                                            _Float16* Y, int ycol, int ytok0, float inv, float osc) {
    const int l = LANE(), i16 = l & 15, g = l >> 4;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        f32x4 v = (hi[ct] + lo[ct] * kLoScale) * inv + bb;
        if (RELU) {
            v.x = relu_nan(v.x); v.y = relu_nan(v.y); v.z = relu_nan(v.z); v.w = relu_nan(v.w);
        }
        hsplit_store(Y, psw((ytok0 + 16 * ct + i16), ycol + 4 * g), v * osc);
    }
}

// Y[ytok0 + 16 ct + j][ycol + i] = epi(acc + bias[brow + i]); lane (j, g) holds rows 4g..4g+3
template <int CT, bool RELU>
__device__ __forceinline__ void store_tile(TID_F const f32x4 (&acc)[CT], const f32x4 bb, float* Y, int ldy, int ycol,
                                           int ytok0) {
    const int l = LANE(), i16 = l & 15, g = l >> 4;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        f32x4 v = acc[ct] + bb;
        if (RELU) {
            v.x = relu_nan(v.x); v.y = relu_nan(v.y); v.z = relu_nan(v.z); v.w = relu_nan(v.w);
        }
        *reinterpret_cast<f32x4*>(Y + (ytok0 + 16 * ct + i16) * ldy + ycol + 4 * g) = v;
    }
}

// One 16-row output tile per wave: Y[tok][ycol + i] = epi(W[row + i] . X[tok]^T + b[row + i]).
// The bias is loaded ahead of the k-loop, so the epilogue does not wait one more L2 round trip.
template <int CT, bool RELU, int D>
__device__ __forceinline__ void linear1(TID_F const APre<D>& pre, const float* W, int ldw, const float* bias, int row,
                                        const float* X, int ldx, int xtok0, float* Y, int ldy, int ycol, int ytok0) {
    const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + row + 4 * (LANE() >> 4));
    f32x4 acc[CT];
    zero(acc);
    gemm_tile<CT, D>(TID_C acc, pre, W, ldw, row, 0, X, ldx, xtok0);
    store_tile<CT, RELU>(TID_C acc, bb, Y, ldy, ycol, ytok0);
}

// ------------------------------------------------------------------ VALU pieces
// Cross-lane sums without the LDS crossbar (__shfl_xor lowers to ds_bpermute on gfx950):
// DPP quad permutes inside a quad, v_permlane16/32_swap across rows / halves. Both lanes of a
// pair compute the same a + b, so the results are bitwise equal across the group.
__device__ __forceinline__ float add_xor1(float v) {
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));  // [1,0,3,2]
}
__device__ __forceinline__ float add_xor2(float v) {
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));  // [2,3,0,1]
}
__device__ __forceinline__ float add_xor16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float add_xor32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// max over each row of 16 lanes (quad permutes, then row_ror 4 / 8), the same in every lane of the row
template <int ctrl>
__device__ __forceinline__ float max_dpp(float v) {
    return fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xF, 0xF, true)));
}
__device__ __forceinline__ float row16_max(float v) {
    return max_dpp<0x128>(max_dpp<0x124>(max_dpp<0x4E>(max_dpp<0xB1>(v))));
}
// max over the wave (the same value in every lane)
__device__ __forceinline__ float wave_max(float v) {
    v = row16_max(v);
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// Fused GEMM epilogue + post-LN (nn.TransformerEncoderLayer norm1 / norm2, eps 1e-5):
//   h[tok][f] = LN(h[tok] + acc + bias)[f] * w[f] + b[f]
// for this wave's 16 output features f = [16 wv, 16 wv + 16) of CT column tiles from ytok0. The
// token statistics combine per-wave (mean, M2) pairs over 16 features each (Chan et al.), so one
// barrier suffices and the variance is two-pass accurate. Ends WITHOUT a barrier after writing h.
// Training-mode outputs of a LayerNorm: normalised rows, output rows, 1/std per row, in the
// workspace layout (compact [b] rows for the pruned tail, [b * 5 + s] rows otherwise).
struct LnOut {
    float *x, *h, *rs;
    int b0, compact;
    bool nt = true;  // non-temporal stores (act_st): not in the position-split kernels
};
__device__ __forceinline__ int trow(int tok, int b0) { return (b0 + (tok & (SPW - 1))) * S + tok / SPW; }
__device__ __forceinline__ int orow(int tok, int b0, bool compact) {
    return compact ? b0 + (tok & (SPW - 1)) : trow(tok, b0);
}

// The epilogue's per-feature operands: the GEMM bias, loaded by the caller BEFORE the GEMM (the
// epilogue's first instruction needs it, so a load issued after the GEMM would expose a whole L2
// round trip), and the LN weight and bias, loaded right after the GEMM -- ahead of its next
// prefetches and the barrier, whose latency then covers them.
struct LnPar {
    f32x4 bb, ww, lb;
};
__device__ __forceinline__ f32x4 ln_bias(TID_F const float* __restrict__ bias) {
    return *reinterpret_cast<const f32x4*>(bias + 16 * (TIDX() >> 6) + 4 * (LANE() >> 4));
}
__device__ __forceinline__ LnPar ln_load(TID_F const f32x4 bb, const float* __restrict__ w, const float* __restrict__ b) {
    const int f0 = 16 * (TIDX() >> 6) + 4 * (LANE() >> 4);
    return LnPar{bb, *reinterpret_cast<const f32x4*>(w + f0), *reinterpret_cast<const f32x4*>(b + f0)};
}
// PLANES: the output goes to sm.h as the two fp16 planes of the split products (the next GEMM's
// operand; the caller keeps the fp32 output from `outv`); resid: the residual from registers (the
// lane's own elements, as `outv` returned them) instead of sm.h.
// ROW4 (with PLANES): the fp32 output of position 4 (tokens 64-79) also goes to sm.ctx rows 0-15 (the
// next, pruned layer's residual and query rows). psc: the planes' scale (the operand's 2^-s).
// T0 / T1 / T2 (trace builds, >= 0): phase stamps when the GEMM accumulators are consumed, when the
// partial statistics are written, after the barrier
template <int CT, bool TR = false, bool PLANES = false, bool ROW4 = false, int T0 = -1, int T1 = -1, int T2 = -1>
__device__ __forceinline__ void residual_layernorm(TID_F Smem& sm, const f32x4 (&acc)[CT], const LnPar& lp, int ytok0,
                                                   const LnOut& lo = LnOut{}, f32x4* outv = nullptr,
                                                   const f32x4* resid = nullptr, float psc = 1.f) {
    const int l = LANE(), i16 = l & 15, g = l >> 4, wv = TIDX() >> 6;
    const int f0 = 16 * wv + 4 * g;
    const f32x4 bb = lp.bb;
    f32x4 v[CT];
#if defined(UAVHIP_POLICY_TRACE)
    if constexpr (T0 >= 0) {
        float dep = 0.f;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) dep += acc[ct].x;
        asm volatile("" ::"v"(dep));
        __builtin_amdgcn_sched_barrier(0);
        PTR(T0);
    }
#endif
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        const int tok = ytok0 + 16 * ct + i16;
        v[ct] = acc[ct] + bb + (resid ? resid[ct] : *reinterpret_cast<const f32x4*>(sm.h + tok * LDH + f0));
        float s = (v[ct].x + v[ct].y) + (v[ct].z + v[ct].w);
        s = add_xor32(add_xor16(s));
        const float m = s * (1.0f / 16);
        const f32x4 d = v[ct] - m;
        float q = (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
        q = add_xor32(add_xor16(q));
        if (g == 0) sm.red[wv * TOK + tok] = make_float2(m, q);
    }
#if defined(UAVHIP_POLICY_TRACE)
    if constexpr (T1 >= 0) {
        __builtin_amdgcn_sched_barrier(0);
        PTR(T1);
    }
#endif
    __syncthreads();
#if defined(UAVHIP_POLICY_TRACE)
    if constexpr (T2 >= 0) PTR(T2);
#endif
    const f32x4 ww = lp.ww, lb = lp.lb;
    // (mean, 1/std) of token tok from the 8 per-wave partials
    auto stats = [&](int tok, float& mean, float& rs) {
        float2 pr[NW];
        float ms = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            pr[k] = sm.red[k * TOK + tok];
            ms += pr[k].x;
        }
        mean = ms * (1.0f / NW);
        float m2 = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const float dm = pr[k].x - mean;
            m2 += pr[k].y + 16.0f * dm * dm;
        }
        rs = ln_rstd(m2 * (1.0f / D) + 1e-5f);
    };
    static_assert(CT == 1 || CT == S, "pruned tile or all five");
    // all five tiles: lane (i16, g) combines the partials of tile g's token, the last tile's in a
    // second round; the other rows of the wave fetch theirs with ds_bpermute (instead of every row
    // of the wave redoing every token's combine)
    float mA, rA, mB, rB;
    if constexpr (CT == 1) stats(ytok0 + i16, mA, rA);
    else {
        stats(ytok0 + 16 * g + i16, mA, rA);
        stats(ytok0 + 16 * (S - 1) + i16, mB, rB);
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        const int tok = ytok0 + 16 * ct + i16;
        float mean = mA, rs = rA;
        if (CT > 1 && ct < S - 1) {
            mean = __shfl(mA, 16 * ct + i16);
            rs = __shfl(rA, 16 * ct + i16);
        } else if (CT > 1) {
            mean = mB;
            rs = rB;
        }
        const f32x4 xh = (v[ct] - mean) * rs;
        const f32x4 out = xh * ww + lb;
        if constexpr (PLANES) hsplit_store(reinterpret_cast<_Float16*>(sm.h), psw(tok, f0), out * psc);
        else *reinterpret_cast<f32x4*>(sm.h + tok * LDH + f0) = out;
        if constexpr (ROW4) {
            if (ct == CT - 1) *reinterpret_cast<f32x4*>(sm.ctx + (tok - (S - 1) * SPW) * LDH + f0) = out;
        }
        if (outv) outv[ct] = out;
        if (TR && !kExpNoStore) {
            const size_t r = (size_t)orow(tok, lo.b0, lo.compact);
            act_st(lo.x + r * D + f0, xh, lo.nt);
            if (lo.h) act_st(lo.h + r * D + f0, out, lo.nt);  // nullptr: formed by k_wgrad
            if (wv == 0 && g == 0) lo.rs[r] = rs;
        }
    }
}

// Training mode: copy [tok][cols] rows from LDS (stride lds) to workspace rows (stride ldo, column
// offset c0) for tokens [t0, t1), all 512 threads, float4 granules.
__device__ __forceinline__ void store_rows(TID_F const float* src, int lds, float* dst, int ldo, int c0, int ncols, int t0,
                                           int b0, bool compact, int t1 = TOK, bool nt = true) {
#ifdef UAVHIP_EXP_NOSTORE  // timing experiment only (make NOSTORE=1): activations not written
    return;
#endif
    const int n4 = ncols / 4, items = (t1 - t0) * n4;
    for (int i = TIDX(); i < items; i += NTHR) {
        const int tok = t0 + i / n4, q = i % n4;
        act_st(dst + (size_t)orow(tok, b0, compact) * ldo + c0 + 4 * q, *reinterpret_cast<const f32x4*>(src + tok * lds + 4 * q), nt);
    }
}

// Full-layer attention for heads [4c, 4c+4): one (sample, head, query group) task per 4 lanes,
// each lane owning 4 of the 16 head dims; the task loads the 5 keys / values once for all its
// queries (group 0: positions 0-2 on waves 0-3, group 1: positions 3-4 on waves 4-7).
// attention_full_core leaves the outputs in registers (o[qi] for query position qs0 + qi, qi < nq);
// attention_full_store writes them to sm.ctx (PLANES: as the split products' fp16 planes).
__device__ __forceinline__ void attention_full_core(TID_F Smem& sm, int c, f32x4 (&o)[3]) {
    const int q4 = TIDX() & 3, task = TIDX() >> 2;
    const int hh = task & 3, p = (task >> 2) & 15, grp = task >> 6;
    const int d0 = hh * HD + 4 * q4;
    f32x4 k[S], v[S];
    bool msk[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
        k[j] = *reinterpret_cast<const f32x4*>(sm.big + (j * SPW + p) * LDB + 64 + d0);
        v[j] = *reinterpret_cast<const f32x4*>(sm.big + (j * SPW + p) * LDB + 128 + d0);
        msk[j] = sm.mask[p * S + j] != 0;
    }
    const int qs0 = grp ? 3 : 0, nq = grp ? 2 : 3;
#pragma unroll
    for (int qi = 0; qi < 3; ++qi) {
        o[qi] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (qi < nq) {
            const int ti = (qs0 + qi) * SPW + p;
            const f32x4 q = *reinterpret_cast<const f32x4*>(sm.big + ti * LDB + d0) * kAttQ;
            float sc[S];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                float part = att_dot(q, k[j]);
                part = add_xor2(add_xor1(part));
                sc[j] = msk[j] ? -INFINITY : part * kAttS;  // 1/sqrt(16)
                mx = j ? fmaxf(mx, sc[j]) : sc[j];
            }
            float den = 0.f;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                sc[j] = __expf(sc[j] - mx);
                den = j ? den + sc[j] : sc[j];
            }
            const float inv = att_recip(den);
            att_mix(o[qi], sc, inv, v);
        }
    }
}
// sc: the planes' scale (PLANES), of this thread's sample p (attn_sc)
template <bool PLANES>
__device__ __forceinline__ void attention_full_store(TID_F Smem& sm, int c, const f32x4 (&o)[3], float sc = 1.f) {
    const int q4 = TIDX() & 3, task = TIDX() >> 2;
    const int hh = task & 3, p = (task >> 2) & 15, grp = task >> 6;
    const int d0 = hh * HD + 4 * q4, qs0 = grp ? 3 : 0, nq = grp ? 2 : 3;
#pragma unroll
    for (int qi = 0; qi < 3; ++qi) {
        if (qi < nq) {
            const int ti = (qs0 + qi) * SPW + p;
            if constexpr (PLANES) hsplit_store(reinterpret_cast<_Float16*>(sm.ctx), psw(ti, 4 * c * HD + d0), o[qi] * sc);
            else *reinterpret_cast<f32x4*>(sm.ctx + ti * LDH + 4 * c * HD + d0) = o[qi];
        }
    }
}
// The planes' scale of an attention output of sample p (1 when it is stored in fp32)
template <bool PLANES, int trunk, int layer>
__device__ __forceinline__ float attn_sc(const Smem& sm, int p) {
    if constexpr (PLANES) return att_sc<trunk, layer>(sm, p).sc;
    else return 1.f;
}
// PLANES: the output goes to sm.ctx as the two fp16 planes of the split products (the out-projection's
// operand), scaled for layer `layer` of trunk `trunk`.
// (no defaults: every call site names the operand whose scale the planes carry -- ADVICE r05)
template <bool PLANES, int trunk, int layer>
__device__ void attention_full(TID_F Smem& sm, int c, const float* __restrict__ P = nullptr) {
    f32x4 o[3];
    attention_full_core(TID_C sm, c, o);
    attention_full_store<PLANES>(TID_C sm, c, o, attn_sc<PLANES, trunk, layer>(sm, (int)((TIDX() >> 4) & 15)));
}

// Scaled-dot-product attention for heads [4c, 4c+4) of the query positions [qs0, qs0 + nqs) over
// the keys/values of all 5 positions; reads sm.big (Q|K|V of the chunk), writes sm.ctx.
// One (query, head) task per 4 consecutive lanes, each lane owning 4 of the 16 head dims
// (dot products reduced over the quad with two xor-shuffles). _core: one query position (nqs = 1):
// threads < 256 own one task each, its output in `o`.
__device__ __forceinline__ void attention_task(TID_F Smem& sm, int task, int qs0, f32x4& o, int& ti, int& d0) {
    const int q4 = TIDX() & 3;
    const int hh = task & 3, rest = task >> 2, p = rest & 15, si = qs0 + (rest >> 4);
    ti = si * SPW + p;
    d0 = hh * HD + 4 * q4;
    const f32x4 q = *reinterpret_cast<const f32x4*>(sm.big + ti * LDB + d0) * kAttQ;
    float sc[S];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < S; ++j) {
        const f32x4 k = *reinterpret_cast<const f32x4*>(sm.big + (j * SPW + p) * LDB + 64 + d0);
        float part = att_dot(q, k);
        part = add_xor2(add_xor1(part));
        sc[j] = sm.mask[p * S + j] ? -INFINITY : part * kAttS;  // 1/sqrt(16)
        mx = j ? fmaxf(mx, sc[j]) : sc[j];
    }
    float den = 0.f;
#pragma unroll
    for (int j = 0; j < S; ++j) {
        sc[j] = __expf(sc[j] - mx);
        den = j ? den + sc[j] : sc[j];
    }
    const float inv = att_recip(den);
    f32x4 v[S];
#pragma unroll
    for (int j = 0; j < S; ++j) v[j] = *reinterpret_cast<const f32x4*>(sm.big + (j * SPW + p) * LDB + 128 + d0);
    o = f32x4{0.f, 0.f, 0.f, 0.f};
    att_mix(o, sc, inv, v);
}
template <bool PLANES>
__device__ __forceinline__ void attention_out(TID_F Smem& sm, int c, int ti, int d0, const f32x4 o, float sc = 1.f) {
    if constexpr (PLANES) hsplit_store(reinterpret_cast<_Float16*>(sm.ctx), psw(ti, 4 * c * HD + d0), o * sc);
    else *reinterpret_cast<f32x4*>(sm.ctx + ti * LDH + 4 * c * HD + d0) = o;
}
template <bool PLANES, int trunk, int layer>
__device__ void attention_chunk(TID_F Smem& sm, int c, int qs0, int nqs, const float* __restrict__ P = nullptr) {
    const int ntask = nqs * SPW * 4;
    for (int task = TIDX() >> 2; task < ntask; task += NTHR / 4) {
        f32x4 o;
        int ti, d0;
        attention_task(TID_C sm, task, qs0, o, ti, d0);
        attention_out<PLANES>(TID_C sm, c, ti, d0, o, attn_sc<PLANES, trunk, layer>(sm, ti & 15));
    }
}

// Embedding (transformer_net.py:57-59) on the MFMA, K = 14 padded to 16 with zeros:
// h[s*16+p][f] = relu(W_e x[p][s] + b_e)[f] + pos[s][f]; wave w computes features [16w, 16w+16).
// The global operands (weights, bias, position rows) are loaded up front (embed_load), so a caller
// can issue later loads behind them without the embedding waiting for those (in-order vmcnt).
struct EmbPre {
    f32x4 a, bb, pp[S];
};
template <int trunk>
__device__ __forceinline__ EmbPre embed_load(TID_F const float* __restrict__ P) {
    const float* We = P + kOffs.o[trunk + EMB_W];
    const float* be = P + kOffs.o[trunk + EMB_B];
    const float* pos = P + kOffs.o[trunk + POS];
    const int l = LANE(), i16 = l & 15, g = l >> 4, wv = TIDX() >> 6;
    const int f = 16 * wv + i16;
    EmbPre r;
    r.a.x = 4 * g + 0 < IN ? We[f * IN + 4 * g + 0] : 0.f;
    r.a.y = 4 * g + 1 < IN ? We[f * IN + 4 * g + 1] : 0.f;
    r.a.z = 4 * g + 2 < IN ? We[f * IN + 4 * g + 2] : 0.f;
    r.a.w = 4 * g + 3 < IN ? We[f * IN + 4 * g + 3] : 0.f;
    r.bb = *reinterpret_cast<const f32x4*>(be + 16 * wv + 4 * g);
#pragma unroll
    for (int ct = 0; ct < S; ++ct) r.pp[ct] = *reinterpret_cast<const f32x4*>(pos + ct * D + 16 * wv + 4 * g);
    return r;
}
// MODE kEmbH: h = e + pos for all 5 positions (sm.h). kEmbSplit: also e of position 4 (no pos)
// -> sm.ctx rows 64-79 (the window-row projection path's in_proj input). kEmbRows: only e of
// positions 0-3 -> sm.ctx (row projection fill).
enum { kEmbH = 0, kEmbSplit = 1, kEmbRows = 2 };
// PL (kEmbH): also the two fp16 planes of h into sm.ctx (the split layer-0 in_proj's operand,
// encoder_layer_split).
template <int trunk, bool TR = false, int MODE = kEmbH, bool PL = false>
__device__ void embed_apply(TID_F Smem& sm, const EmbPre& ep, float* e_out = nullptr, float* h_out = nullptr, int b0 = 0) {
    const int l = LANE(), i16 = l & 15, g = l >> 4, wv = TIDX() >> 6;
    constexpr int NT = MODE == kEmbRows ? S - 1 : S;
    // the ring forward's actor (its only layer is pruned to position 4): positions 0-3 come from the
    // ring rows and only position 4 is a residual, so only its embedding is formed
    constexpr int CT0 = MODE == kEmbSplit && trunk == kActorTrunk ? S - 1 : 0;
    f32x4 acc[NT];
#pragma unroll
    for (int ct = CT0; ct < NT; ++ct) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(sm.x + (ct * SPW + i16) * LDX + 4 * g);
        acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(ep.a[j], b[j], acc[ct], 0, 0, 0);
    }
#pragma unroll
    for (int ct = CT0; ct < NT; ++ct) {
        f32x4 e = acc[ct] + ep.bb;
        e.x = fmaxf(e.x, 0.f); e.y = fmaxf(e.y, 0.f); e.z = fmaxf(e.z, 0.f); e.w = fmaxf(e.w, 0.f);
        const int o = (ct * SPW + i16) * LDH + 16 * wv + 4 * g;
        constexpr bool ring_planes = split_slot(layer_param(trunk, 0, INW)) >= 0;  // the ring GEMM's operand
        // the planes of layer 0's input scaled per token (its window row's range)
        const float esc = (ring_planes || PL) ? es_factor<trunk, -1>(sm, ct * SPW + i16) : 1.f;
        if ((MODE == kEmbRows || (MODE == kEmbSplit && ct == S - 1)) && ring_planes)
            hsplit_store(reinterpret_cast<_Float16*>(sm.ctx), psw((ct * SPW + i16), 16 * wv + 4 * g), e * esc);
        else if (MODE == kEmbRows || (MODE == kEmbSplit && ct == S - 1)) *reinterpret_cast<f32x4*>(sm.ctx + o) = e;
        if (MODE == kEmbRows) continue;
        const f32x4 v = e + ep.pp[ct];
        *reinterpret_cast<f32x4*>(sm.h + o) = v;
        if constexpr (PL) hsplit_store(reinterpret_cast<_Float16*>(sm.ctx), psw((ct * SPW + i16), 16 * wv + 4 * g), v * esc);
        if (TR && !kExpNoStore) {
            const size_t r = (size_t)trow(ct * SPW + i16, b0);
            act_st(e_out + r * D + 16 * wv + 4 * g, e);
            if (h_out) act_st(h_out + r * D + 16 * wv + 4 * g, v);
        }
    }
}
template <int trunk, bool TR = false>
__device__ void embed(TID_F Smem& sm, const float* __restrict__ P, float* e_out = nullptr, float* h_out = nullptr,
                      int b0 = 0) {
    embed_apply<trunk, TR>(TID_C sm, embed_load<trunk>(TID_C P), e_out, h_out, b0);
}

// K/V weight row of wave wv for chunk c: waves 0-3 K tiles, waves 4-7 V tiles
__device__ __forceinline__ int kv_row(int wv, int c) { return (1 + (wv >> 2)) * D + 64 * c + 16 * (wv & 3); }

// A caller's hook run inside layer_tail after the FFN2 GEMM, before the LN2 epilogue (training
// mode: the next phase's global loads issued ahead of LN2's activation stores -- the vector memory
// counter retires in order, so a load behind a store burst waits for the whole burst).
struct NoHook {
    __device__ void operator()() const {}
};
// Split-product paths of the inference forward (policy_layout.hpp kSplitParam): a full layer whose
// out-projection and FFN run on the f16 cores, and a layer whose in_proj does (K / V / Q from the
// fp16 planes of its input, which the previous layer's LN2 then writes).
template <int trunk, int layer>
constexpr bool split_tail() {
    return layer < 2 && split_slot(layer_param(trunk, layer, OUTW)) >= 0 && split_slot(layer_param(trunk, layer, L1W)) >= 0 &&
           split_slot(layer_param(trunk, layer, L2W)) >= 0;
}
template <int trunk, int layer>
constexpr bool split_inproj() {  // layer >= 1: its input comes from a split full layer's LN2 (layer 0's
                                 // in_proj split copy serves the window-row ring only: split_ring)
    return layer >= 1 && layer < 2 && split_slot(layer_param(trunk, layer, INW)) >= 0;
}
// The caller's prefetch of a layer tail's first out-projection weights / of a layer's first K/V
// weights: the split copy's blocks on the split paths, the fp32 fragments otherwise. SP selects the
// split paths: the inference forward always (SP = !TR), the training forward (TR) when its caller
// asks (kTrainSplit); the position-split kernels (PSX) never.
template <int trunk, int layer>
constexpr bool split_l0() {  // layer 0's in_proj from the embedding's planes (the training forward)
    return layer == 0 && split_slot(layer_param(trunk, 0, INW)) >= 0;
}
// Weight blocks (of 32 k) a split tail GEMM has in registers before its k-loop starts: the pruned
// (one 16-token tile) tails of the inference forward take their whole tile (4 blocks) -- their MFMA
// work per block is a fifth of a full layer's, far too little to cover an in-loop L2 round trip --
// the rest 2 (EXP=74: the A/B build of the full-tile prefetch)
constexpr bool kExpTailDepth4 = UAVHIP_EXP == 74;
template <bool last, bool TR, int PSX>
constexpr int tail_depth() { return kExpTailDepth4 && last && !TR && !PSX ? 4 : 2; }
template <int trunk, int layer, bool last, bool TR, int PSX = 0, bool SP = !TR>
using TailPre = std::conditional_t<SP && !PSX && split_tail<trunk, layer>(), HPre<tail_depth<last, TR, PSX>()>,
                                   APre<depth<(last || PSX) ? 1 : S>()>>;
template <int trunk, int layer, bool last, bool TR, bool SP = !TR>
__device__ __forceinline__ TailPre<trunk, layer, last, TR, 0, SP> tail_prefetch(TID_F const float* __restrict__ P) {
    const int wv = TIDX() >> 6;
    if constexpr (SP && split_tail<trunk, layer>())
        return hprefetch<tail_depth<last, TR, 0>()>(TID_C P, split_slot(layer_param(trunk, layer, OUTW)), D, 16 * wv, 0);
    else
        return prefetch<depth<last ? 1 : S>()>(TID_C P + kOffs.o[layer_param(trunk, layer, OUTW)], D, 16 * wv, 0);
}
template <int trunk, int layer, bool TR, bool SP = !TR>
constexpr bool split_kv() {
    return SP && (split_inproj<trunk, layer>() || (TR && split_l0<trunk, layer>()));
}
template <int trunk, int layer, bool TR, bool SP = !TR>
using KvPre = std::conditional_t<split_kv<trunk, layer, TR, SP>(), HPre<2>, APre<2>>;
template <int trunk, int layer, bool TR, bool SP = !TR>
__device__ __forceinline__ KvPre<trunk, layer, TR, SP> kv_prefetch(TID_F const float* __restrict__ P) {
    const int wv = TIDX() >> 6;
    if constexpr (split_kv<trunk, layer, TR, SP>())
        return hprefetch<2>(TID_C P, split_slot(layer_param(trunk, layer, INW)), D, kv_row(wv, 0), 0);
    else
        return prefetch<2>(TID_C P + kOffs.o[layer_param(trunk, layer, INW)], D, kv_row(wv, 0), 0);
}
// The training forward's split switch (k_policy_forward<true>; the K7 kernels: kPsSplit below).
constexpr bool kTrainSplit = true;

// PSX (position split, the small-minibatch training step): a full (unpruned) layer computed for
// the 16 tokens of ONE window position, column tile qt / 16, in [b * 5 + s] rows.
template <int trunk, int layer, bool last, bool TR, class F = NoHook, int PSX = 0, bool SP = !TR>
__device__ __forceinline__ void layer_tail(TID_F Smem& sm, const float* __restrict__ P, const TailPre<trunk, layer, last, TR, PSX, SP>& po,
                           const TrainLayerIO& io, int b0, F pre_ln2 = F{}, int qt = 0);

// Training mode: the Q|K|V of chunk c of the tokens [qtok0, 80) (Q) / all (K, V) from sm.big to qkv
// rows, by waves 4-7 (less MFMA work than the K + Q waves sharing their SIMDs).
// EXP=81 (timing only, WRONG results): the Q | K | V stream between the training forward and K6
// compiled out -- the forward does not store it, K6 reads one hot row for every sample (the ceiling
// of recomputing it in K6, DESIGN.md 10 lever 3)
constexpr bool kExpNoQkvStream = UAVHIP_EXP == 81;
__device__ __forceinline__ void store_qkv_chunk(TID_F const Smem& sm, float* __restrict__ qkv, int c, int qtok0, int b0) {
    if (kExpNoStore || kExpNoQkvStream) return;
    for (int i = (int)TIDX() - NTHR / 2; i < TOK * 48; i += NTHR / 2) {
        if (i < 0) break;
        const int tok = i / 48, r = i - tok * 48, part = r >> 4, q = r & 15;
        if (part == 0 && tok < qtok0) continue;
        act_st(qkv + (size_t)trow(tok, b0) * 3 * D + part * D + 64 * c + 4 * q,
               *reinterpret_cast<const f32x4*>(sm.big + tok * LDB + part * 64 + 4 * q));
    }
}
// Training mode: fp32 rows from the two planes of a split-product operand in LDS (the values the
// GEMM consumed: (x1 + 2^-11 x2) 2^s, inv(tok) = 2^s of the token's operand scale) -> workspace rows
// (stride ldo, column offset c0), tokens [t0, t1).
template <class Inv>
__device__ __forceinline__ void store_rows_planes(TID_F const _Float16* src, float* dst, int ldo, int c0, int ncols,
                                                  int t0, int b0, bool compact, int t1, Inv inv, bool nt = true) {
    if (kExpNoStore) return;
    const int n4 = ncols / 4, items = (t1 - t0) * n4;
    for (int i = TIDX(); i < items; i += NTHR) {
        const int tok = t0 + i / n4, q = i % n4;
        const f16x4 x1 = *reinterpret_cast<const f16x4*>(src + psw(tok, 4 * q));
        const f16x4 x2 = *reinterpret_cast<const f16x4*>(src + kPlane + psw(tok, 4 * q));
        const float s = inv(tok);
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = ((float)x1[j] + (float)x2[j] * kLoScale) * s;
        act_st(dst + (size_t)orow(tok, b0, compact) * ldo + c0 + 4 * q, v, nt);
    }
}

// 2^s of a layer's in_proj operand at token tok: layer 0's input per token (its window row's range),
// a later layer's input = the previous layer's LN2 output (static)
template <int trunk, int layer>
__device__ __forceinline__ float in_inv(const Smem& sm, int tok) {
    if constexpr (layer == 0) return es_factor<trunk, 1>(sm, tok);
    else return op_sc<trunk, layer - 1, kOpLn2>(sm).inv;
}

// An encoder layer whose in_proj runs as split products: K / V of all 80 tokens and Q of the query
// tokens from the fp16 planes of the layer input, fp32 Q | K | V into sm.big, then attention and
// the layer tail. The input planes are
//   layer >= 1: in sm.h (the previous layer's LN2 wrote them, and its position-4 rows in fp32 to
//               sm.ctx rows 0-15: the residual of this pruned layer);
//   layer 0 (training forward): in sm.ctx (the embedding wrote them beside its fp32 rows in sm.h) --
//               so chunk 0's attention output waits in registers until chunk 1's GEMMs have read
//               sm.ctx, then both chunks are written.
template <int trunk, int layer, bool last, bool TR, class F = NoHook>
__device__ __forceinline__ void encoder_layer_split(TID_F Smem& sm, const float* __restrict__ P, HPre<2> pkv,
                                                    const TrainLayerIO& io, int b0, F pre_ln2) {
    [[maybe_unused]] constexpr int tb = 8 + 16 * (trunk == 0 ? 0 : 1 + layer);  // trace slot base
    PTR(tb);
    constexpr int si = split_slot(layer_param(trunk, layer, INW));
    constexpr int CTQ = last ? 1 : S, qtok0 = last ? (S - 1) * SPW : 0;
    constexpr bool in_ctx = layer == 0;                 // the input planes: sm.ctx (layer 0) or sm.h
    constexpr bool planes = split_tail<trunk, layer>();  // the attention output as planes
    static_assert(in_ctx || last, "a split in_proj after a split full layer: a pruned layer");
    const float* bin = P + kOffs.o[layer_param(trunk, layer, INB)];
    const int l = LANE(), i16 = l & 15, g = l >> 4, wv = TIDX() >> 6;
    const _Float16* hp = reinterpret_cast<const _Float16*>(in_ctx ? sm.ctx : sm.h);
    TailPre<trunk, layer, last, TR, 0, true> po;
    [[maybe_unused]] f32x4 att0[last ? 1 : 3];  // chunk 0's attention output (in_ctx)
    [[maybe_unused]] int ti0 = 0, d00 = 0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {  // two chunks of 4 heads (LDS budget)
        HPre<2> pq;
        if (wv < 4) pq = hprefetch<2>(TID_C P, si, D, 64 * c + 16 * wv, 0);
        {  // K (waves 0-3) / V (waves 4-7) of the chunk for all 80 tokens
            const f32x4 bb = *reinterpret_cast<const f32x4*>(bin + kv_row(wv, c) + 4 * g);
            f32x4 hi[S], lo[S];
            zero(hi);
            zero(lo);
            hgemm_tile<S, 2>(TID_C hi, lo, pkv, P, si, D, kv_row(wv, c), 0, hp, 0);
            if constexpr (layer == 0) __asm__ volatile("" ::: "memory");  // the scales' LDS reads after the GEMM
            const int col = (1 + (wv >> 2)) * 64 + 16 * (wv & 3) + 4 * g;
#pragma unroll
            for (int ct = 0; ct < S; ++ct)
                *reinterpret_cast<f32x4*>(sm.big + (16 * ct + i16) * LDB + col) =
                    (hi[ct] + lo[ct] * kLoScale) * in_inv<trunk, layer>(sm, 16 * ct + i16) + bb;
        }
        if (wv < 4) {  // Q of the chunk for the query tokens (their SIMD partners did V)
            const f32x4 bq = *reinterpret_cast<const f32x4*>(bin + 64 * c + 16 * wv + 4 * g);
            f32x4 hi[CTQ], lo[CTQ];
            zero(hi);
            zero(lo);
            hgemm_tile<CTQ, 2>(TID_C hi, lo, pq, P, si, D, 64 * c + 16 * wv, 0, hp, qtok0);
            if constexpr (layer == 0) __asm__ volatile("" ::: "memory");
#pragma unroll
            for (int ct = 0; ct < CTQ; ++ct)
                *reinterpret_cast<f32x4*>(sm.big + (qtok0 + 16 * ct + i16) * LDB + 16 * wv + 4 * g) =
                    (hi[ct] + lo[ct] * kLoScale) * in_inv<trunk, layer>(sm, qtok0 + 16 * ct + i16) + bq;
        }
        if (c == 0) pkv = hprefetch<2>(TID_C P, si, D, kv_row(wv, 1), 0);
        else po = tail_prefetch<trunk, layer, last, TR, true>(TID_C P);
        PTR(tb + 1 + 3 * c);
        __syncthreads();
        PTR(tb + 2 + 3 * c);
        if constexpr (TR) store_qkv_chunk(TID_C sm, io.qkv, c, qtok0, b0);
        if constexpr (!in_ctx) {
            attention_chunk<planes, trunk, layer>(TID_C sm, c, S - 1, 1, P);
        } else if constexpr (last) {  // one query position: threads < 256 own one task each
            f32x4 o;
            int ti = 0, d0 = 0;
            if (TIDX() < 4 * SPW * 4) attention_task(TID_C sm, TIDX() >> 2, S - 1, o, ti, d0);
            if (c == 0) {
                att0[0] = o;
                ti0 = ti;
                d00 = d0;
            } else if (TIDX() < 4 * SPW * 4) {
                const float asc = attn_sc<planes, trunk, layer>(sm, ti & 15);
                attention_out<planes>(TID_C sm, 0, ti0, d00, att0[0], asc);
                attention_out<planes>(TID_C sm, 1, ti, d0, o, asc);
            }
        } else {
            if (c == 0) {
                attention_full_core(TID_C sm, 0, att0);
            } else {
                f32x4 o[3];
                attention_full_core(TID_C sm, 1, o);
                const float asc = attn_sc<planes, trunk, layer>(sm, (int)((TIDX() >> 4) & 15));
                attention_full_store<planes>(TID_C sm, 0, att0, asc);
                attention_full_store<planes>(TID_C sm, 1, o, asc);
            }
        }
        __syncthreads();
        PTR(tb + 3 + 3 * c);
    }
    layer_tail<trunk, layer, last, TR, F, 0, true>(TID_C sm, P, po, io, b0, pre_ln2);
}

// One post-LN nn.TransformerEncoderLayer (relu FFN 256, 8 heads). last: prune to column tile 4.
// Work split: 8 waves, wave w and w+4 share a SIMD (and its MFMA pipe); every GEMM gives each
// SIMD the same number of 16-row output tiles. `pkv` = the caller's prefetch of this layer's first
// K/V weight blocks. Ends WITHOUT a final barrier: the caller prefetches its next weights, then syncs.
template <int trunk, int layer, bool last, bool TR = false, class F = NoHook, bool SP = !TR>
__device__ __forceinline__ void encoder_layer(TID_F Smem& sm, const float* __restrict__ P, KvPre<trunk, layer, TR, SP> pkv,
                              const TrainLayerIO& io = TrainLayerIO{}, int b0 = 0, F pre_ln2 = F{}) {
    if constexpr (split_kv<trunk, layer, TR, SP>()) {
        encoder_layer_split<trunk, layer, last, TR, F>(TID_C sm, P, pkv, io, b0, pre_ln2);
        return;
    } else {
    [[maybe_unused]] constexpr int tb = 8 + 16 * (trunk == 0 ? 0 : 1 + layer);  // trace slot base
    PTR(tb);
    const float* Win = P + kOffs.o[layer_param(trunk, layer, INW)];
    const float* bin = P + kOffs.o[layer_param(trunk, layer, INB)];
    const int wv = TIDX() >> 6;
    constexpr int CTQ = last ? 1 : S;              // column tiles that need Q / out / LN / FFN
    constexpr int DQ = depth<CTQ>();
    constexpr int qtok0 = last ? (S - 1) * SPW : 0;
    constexpr bool planes = SP && split_tail<trunk, layer>();

    TailPre<trunk, layer, last, TR, 0, SP> po;
#pragma unroll
    for (int c = 0; c < 2; ++c) {  // two chunks of 4 heads (LDS budget)
        APre<DQ> pq;
        if (wv < 4) pq = prefetch<DQ>(TID_C Win, D, 64 * c + 16 * wv, 0);
        // K (waves 0-3) / V (waves 4-7) of the chunk for all 80 tokens, one 16-row tile each
        linear1<S, false, 2>(TID_C pkv, Win, D, bin, kv_row(wv, c), sm.h, LDH, 0, sm.big, LDB, (1 + (wv >> 2)) * 64 + 16 * (wv & 3), 0);
        // Q of the chunk for the query tokens, waves 0-3 (their SIMD partners did V)
        if (wv < 4) linear1<CTQ, false, DQ>(TID_C pq, Win, D, bin, 64 * c + 16 * wv, sm.h, LDH, qtok0, sm.big, LDB, 16 * wv, qtok0);
        if (c == 0) pkv = prefetch<2>(TID_C Win, D, kv_row(wv, 1), 0);
        else po = tail_prefetch<trunk, layer, last, TR, SP>(TID_C P);
        PTR(tb + 1 + 3 * c);
        __syncthreads();
        PTR(tb + 2 + 3 * c);
        if (TR && !kExpNoStore && !kExpNoQkvStream) {  // this chunk's Q (query tokens) / K / V -> qkv[row][part * 128 + 64 c + d]
            // by waves 4-7 (V tiles: less MFMA work than the K + Q waves sharing their SIMDs)
            for (int i = (int)TIDX() - NTHR / 2; i < TOK * 48; i += NTHR / 2) {
                if (i < 0) break;
                const int tok = i / 48, r = i - tok * 48, part = r >> 4, q = r & 15;
                if (part == 0 && tok < qtok0) continue;
                act_st(io.qkv + (size_t)trow(tok, b0) * 3 * D + part * D + 64 * c + 4 * q,
                       *reinterpret_cast<const f32x4*>(sm.big + tok * LDB + part * 64 + 4 * q));
            }
        }
        if (last) attention_chunk<planes, trunk, layer>(TID_C sm, c, S - 1, 1, P);
        else attention_full<planes, trunk, layer>(TID_C sm, c, P);
        __syncthreads();
        PTR(tb + 3 + 3 * c);
    }
    layer_tail<trunk, layer, last, TR, F, 0, SP>(TID_C sm, P, po, io, b0, pre_ln2);
    }
}

// Out-projection + LN1 + FFN + LN2 of an inference layer as split products (layer_tail's split
// path): a full layer (80 tokens) or a pruned one (the 16 tokens of position 4). The attention
// output's planes are in sm.ctx (attention_full / attention_chunk <true>); LN1 writes its output's
// planes into sm.h and keeps the fp32 values in registers (LN2's residual); FFN1 writes the hidden
// planes into big (features 0-127) and ctx (128-255); LN2 writes fp32 into sm.h -- or, when the next
// layer's in_proj runs as split products, that layer's operand planes (and position 4 in fp32 to
// sm.ctx rows 0-15). A pruned layer after such a layer takes its residual from sm.ctx rows 0-15.
// Training mode (TR): the activations the backward reads are written as in layer_tail -- the
// attention output and the FFN hidden from their planes (the values the GEMMs consumed), the
// LayerNorm outputs from registers.
// PSX (the K7 position-split forward): a full layer for the 16 tokens of one position, [qt, qt + 16),
// its residual in sm.h, LN2's output as planes for the kernel's next in_proj (ps_inproj_split); and
// K7's pruned layers take their residual from sm.h (PSX = 2).
template <int trunk, int layer, bool last, bool TR = false, class F = NoHook, int PSX = 0>
__device__ __forceinline__ void layer_tail_split(TID_F Smem& sm, const float* __restrict__ P,
                                                 const HPre<tail_depth<last, TR, PSX>()>& po,
                                                 const TrainLayerIO& io = TrainLayerIO{}, int b0 = 0, F pre_ln2 = F{},
                                                 int qt = 0) {
    constexpr int DP = tail_depth<last, TR, PSX>();
    [[maybe_unused]] constexpr int tb = 8 + 16 * (trunk == 0 ? 0 : 1 + layer);  // trace slot base
    constexpr int CT = (last || PSX) ? 1 : S;
    const int t0 = last ? (S - 1) * SPW : (PSX ? qt : 0), t1 = t0 + SPW * CT;
    const float* bo = P + kOffs.o[layer_param(trunk, layer, OUTB)];
    const float* b1 = P + kOffs.o[layer_param(trunk, layer, L1B)];
    const float* b2 = P + kOffs.o[layer_param(trunk, layer, L2B)];
    constexpr int s1 = split_slot(layer_param(trunk, layer, L1W)), s2 = split_slot(layer_param(trunk, layer, L2W));
    constexpr int so = split_slot(layer_param(trunk, layer, OUTW));
    // LN2 writes the next layer's operand planes (+ position 4 in fp32 to sm.ctx rows 0-15 for the
    // full forward's pruned next layer)
    constexpr bool next_planes = !last && split_inproj<trunk, layer + 1>();
    constexpr bool row4 = next_planes && !PSX;
    constexpr bool res_ctx = split_inproj<trunk, layer>() && !PSX;  // the residual is in sm.ctx rows 0-15
    static_assert(!res_ctx || last, "a split in_proj feeds a pruned layer");
    constexpr bool kC0 = trunk != 0 && layer == 0 && !TR && !PSX;  // trace stamps of the critic's layer-0 LNs
    const int wv = TIDX() >> 6;
    _Float16* const hp = reinterpret_cast<_Float16*>(sm.h);
    _Float16* const bp = reinterpret_cast<_Float16*>(sm.big);
    _Float16* const cp = reinterpret_cast<_Float16*>(sm.ctx);
    f32x4 h1[CT];  // LN1's output: LN2's residual
    HPre<DP> w1a;
    // the operand scales (policy_layout.hpp range table): the attention output (layer 0: one per
    // workgroup, att_sc), LN1's output, the FFN hidden units; LN2's output when it is the next layer's
    // split operand
    const OpSc s_ln1 = op_sc<trunk, layer, kOpLn1>(sm), s_hid = op_sc<trunk, layer, kOpHid>(sm);
    if constexpr (TR)  // attention output
        store_rows_planes(TID_C cp, io.o, D, 0, D, t0, b0, last, t1,
                          [&](int tok) { return att_sc<trunk, layer>(sm, tok & 15).inv; }, !PSX);
    {
        // the epilogue's bias and LN1's weight / bias ahead of the GEMM: issued after it, their L2
        // round trip (~2 k cycles with every CU reading the same lines) outlasted the partials +
        // barrier + statistics in front of their first use
        const LnPar lp = ln_load(TID_C ln_bias(TID_C bo), P + kOffs.o[layer_param(trunk, layer, N1W)],
                                 P + kOffs.o[layer_param(trunk, layer, N1B)]);
        f32x4 acc[CT];
        {  // out-projection from the attention output's planes
            f32x4 hi[CT], lo[CT];
            zero(hi);
            zero(lo);
            hgemm_tile<CT, DP>(TID_C hi, lo, po, P, so, D, 16 * wv, 0, cp, t0);
            const float att_inv = att_sc<trunk, layer>(sm, LANE() & 15).inv;  // uniform (SGPRs)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) acc[ct] = (hi[ct] + lo[ct] * kLoScale) * att_inv;
        }
        PTR(tb + 7);
        w1a = hprefetch<DP>(TID_C P, s1, D, 16 * wv, 0);
        // the LayerNorm outputs go to the workspace only for the position-split kernels (K7 reads
        // them across launches); the fused training step's weight gradients form them from x-hat
        const LnOut lo1{io.xhat1, PSX ? io.h1 : nullptr, io.rstd1, b0, last, !PSX};
        if constexpr (res_ctx) {
            const f32x4 r4[1] = {*reinterpret_cast<const f32x4*>(sm.ctx + (LANE() & 15) * LDH + 16 * wv + 4 * (LANE() >> 4))};
            residual_layernorm<CT, TR, true>(TID_C sm, acc, lp, t0, lo1, h1, r4, s_ln1.sc);
        } else {
            residual_layernorm<CT, TR, true, false, kC0 ? 55 : -1, kC0 ? 56 : -1, kC0 ? 57 : -1>(TID_C sm, acc, lp, t0, lo1, h1,
                                                                                            nullptr, s_ln1.sc);
        }
    }
    PTR(tb + 8);
    __syncthreads();
    PTR(tb + 9);
    {  // FFN1: hidden features 0-127 -> big planes, 128-255 -> ctx planes (both free now)
        const int grow = 4 * (LANE() >> 4);
        const f32x4 ba = *reinterpret_cast<const f32x4*>(b1 + 16 * wv + grow);
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b1 + 128 + 16 * wv + grow);
        f32x4 hi[CT], lo[CT];
        zero(hi);
        zero(lo);
        // FFN1's second tile's first blocks load under the first tile's last MFMAs (EXP=96: after it)
        HPre<DP> w1b;
        if constexpr (UAVHIP_EXP != 96) {
            hgemm_tile<CT, DP, D / 32, LDP, kPlane, true>(TID_C hi, lo, w1a, P, s1, D, 16 * wv, 0, hp, t0, &w1b,
                                                          hfrag_ptr(TID_C P, s1, D, 128 + 16 * wv, 0));
        } else {
            hgemm_tile<CT, DP>(TID_C hi, lo, w1a, P, s1, D, 16 * wv, 0, hp, t0);
            w1b = hprefetch<DP>(TID_C P, s1, D, 128 + 16 * wv, 0);
        }
        hstore_tile<CT, true>(TID_C hi, lo, ba, bp, 16 * wv, t0, s_ln1.inv, s_hid.sc);
        zero(hi);
        zero(lo);
        hgemm_tile<CT, DP>(TID_C hi, lo, w1b, P, s1, D, 128 + 16 * wv, 0, hp, t0);
        hstore_tile<CT, true>(TID_C hi, lo, bb, cp, 16 * wv, t0, s_ln1.inv, s_hid.sc);
    }
    const HPre<DP> w2a = hprefetch<DP>(TID_C P, s2, FF, 16 * wv, 0);
    PTR(tb + 10);
    __syncthreads();
    PTR(tb + 11);
    const HPre<DP> w2b = hprefetch<DP>(TID_C P, s2, FF, 16 * wv, 128);
    if constexpr (TR) {  // FFN hidden (post-ReLU): features 0-127 from big, 128-255 from ctx
        store_rows_planes(TID_C bp, io.u, FF, 0, D, t0, b0, last, t1, [&](int) { return s_hid.inv; }, !PSX);
        store_rows_planes(TID_C cp, io.u, FF, D, D, t0, b0, last, t1, [&](int) { return s_hid.inv; }, !PSX);
    }
    const LnPar lp2 = ln_load(TID_C ln_bias(TID_C b2), P + kOffs.o[layer_param(trunk, layer, N2W)],
                              P + kOffs.o[layer_param(trunk, layer, N2B)]);  // ahead of the GEMM, as LN1's
    f32x4 hi[CT], lo[CT];
    zero(hi);
    zero(lo);
    hgemm_tile<CT, DP>(TID_C hi, lo, w2a, P, s2, FF, 16 * wv, 0, bp, t0);
    hgemm_tile<CT, DP>(TID_C hi, lo, w2b, P, s2, FF, 16 * wv, 128, cp, t0);
    PTR(tb + 12);
    f32x4 acc2[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc2[ct] = (hi[ct] + lo[ct] * kLoScale) * s_hid.inv;
    pre_ln2();
    float ln2_sc = 1.f;
    if constexpr (next_planes) ln2_sc = op_sc<trunk, layer, kOpLn2>(sm).sc;
    residual_layernorm<CT, TR, next_planes, row4, kC0 ? 23 : -1, kC0 ? 39 : -1, kC0 ? 58 : -1>(
        TID_C sm, acc2, lp2, t0, LnOut{io.xhat2, PSX ? io.h2 : nullptr, io.rstd2, b0, last, !PSX}, nullptr, h1, ln2_sc);
    PTR(tb + 14);
}

// Out-projection + LN1 + FFN + LN2 of an encoder layer, after the attention output is in sm.ctx.
// `po` = the caller's prefetch of the first out_proj weight blocks.
template <int trunk, int layer, bool last, bool TR, class F, int PSX, bool SP>
__device__ __forceinline__ void layer_tail(TID_F Smem& sm, const float* __restrict__ P, const TailPre<trunk, layer, last, TR, PSX, SP>& po,
                           const TrainLayerIO& io, int b0, F pre_ln2, int qt) {
    [[maybe_unused]] constexpr int tb = 8 + 16 * (trunk == 0 ? 0 : 1 + layer);  // trace slot base
    const float* Wo = P + kOffs.o[layer_param(trunk, layer, OUTW)];
    const float* bo = P + kOffs.o[layer_param(trunk, layer, OUTB)];
    const float* W1 = P + kOffs.o[layer_param(trunk, layer, L1W)];
    const float* b1 = P + kOffs.o[layer_param(trunk, layer, L1B)];
    const float* W2 = P + kOffs.o[layer_param(trunk, layer, L2W)];
    const float* b2 = P + kOffs.o[layer_param(trunk, layer, L2B)];
    const int wv = TIDX() >> 6;
    constexpr int CTQ = (last || PSX) ? 1 : S;
    constexpr int DQ = depth<CTQ>();
    const int qtok0 = last ? (S - 1) * SPW : (PSX ? qt : 0);
    const int qtok1 = qtok0 + SPW * CTQ;
    if (TR) store_rows(TID_C sm.ctx, LDH, io.o, D, 0, D, qtok0, b0, last, qtok1, !PSX);  // attention output
    // out projection, h = LN1(h + attn) in its epilogue
    APre<DQ> pf1a, pf1b;
    // inference, full layer (the critic's layer 0): the FFN runs as split products on the f16
    // matrix cores (hgemm_tile): LN1 writes its output as the two fp16 planes into sm.h and keeps
    // the fp32 values in registers (LN2's residual), FFN1 writes the hidden planes into big
    // (features 0-127) and ctx (128-255), FFN2 reads them
    if constexpr (SP && !PSX && split_tail<trunk, layer>()) {
        layer_tail_split<trunk, layer, last, TR, F>(TID_C sm, P, po, io, b0, pre_ln2);
        return;
    } else {
    // a pruned layer after a split full layer: the residual (its input at position 4) is in sm.ctx
    // rows 0-15 (sm.h holds the input's fp16 planes)
    constexpr bool kResCtx = SP && last && !PSX && split_inproj<trunk, layer>();
    // inference, full layer: the wave's own 16 LayerNorm output features are FFN1's k-block wv, so
    // its MFMAs over that block run from registers before the barrier (beside the other waves'
    // LayerNorm work) and the GEMM after it covers the other 7 blocks (k-block order rotated)
    constexpr bool kRot = !TR && CTQ == S;
    [[maybe_unused]] APre<1> own_a, own_b;
    [[maybe_unused]] f32x4 fa[CTQ], fb[CTQ];
    {
        const f32x4 bo4 = ln_bias(TID_C bo);
        f32x4 acc[CTQ];
        zero(acc);
        gemm_tile<CTQ, DQ>(TID_C acc, po, Wo, D, 16 * wv, 0, sm.ctx, LDH, qtok0);
        PTR(tb + 7);
        const LnPar lp = ln_load(TID_C bo4, P + kOffs.o[layer_param(trunk, layer, N1W)], P + kOffs.o[layer_param(trunk, layer, N1B)]);
        if constexpr (kRot) {
            own_a = prefetch_rot<1>(TID_C W1, D, 16 * wv, wv);
            own_b = prefetch_rot<1>(TID_C W1, D, 128 + 16 * wv, wv);
            pf1a = prefetch_rot<DQ>(TID_C W1, D, 16 * wv, wv + 1);
            pf1b = prefetch_rot<DQ>(TID_C W1, D, 128 + 16 * wv, wv + 1);
            f32x4 outv[CTQ];
            residual_layernorm<CTQ, TR>(TID_C sm, acc, lp, qtok0, LnOut{io.xhat1, PSX ? io.h1 : nullptr, io.rstd1, b0, last, !PSX}, outv);
            zero(fa);
            zero(fb);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int ct = 0; ct < CTQ; ++ct) {
                    fa[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(own_a.a[0][j], outv[ct][j], fa[ct], 0, 0, 0);
                    fb[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(own_b.a[0][j], outv[ct][j], fb[ct], 0, 0, 0);
                }
        } else {
            pf1a = prefetch<DQ>(TID_C W1, D, 16 * wv, 0);
            pf1b = prefetch<DQ>(TID_C W1, D, 128 + 16 * wv, 0);
            if constexpr (kResCtx) {
                const f32x4 r4[1] = {*reinterpret_cast<const f32x4*>(sm.ctx + (LANE() & 15) * LDH + 16 * wv + 4 * (LANE() >> 4))};
                residual_layernorm<CTQ, TR>(TID_C sm, acc, lp, qtok0, LnOut{}, nullptr, r4);
            } else {
                residual_layernorm<CTQ, TR>(TID_C sm, acc, lp, qtok0, LnOut{io.xhat1, PSX ? io.h1 : nullptr, io.rstd1, b0, last, !PSX});
            }
        }
    }
    PTR(tb + 8);
    __syncthreads();
    PTR(tb + 9);
    // FFN: hidden features 0-127 -> big, 128-255 -> ctx (both free now), then one K=256 GEMM
    if constexpr (kRot) {
        const int grow = 4 * (LANE() >> 4);
        const f32x4 ba = *reinterpret_cast<const f32x4*>(b1 + 16 * wv + grow);
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b1 + 128 + 16 * wv + grow);
        gemm_tile_rot<CTQ, DQ>(TID_C fa, pf1a, W1, D, 16 * wv, sm.h, LDH, qtok0, wv + 1);
        store_tile<CTQ, true>(TID_C fa, ba, sm.big, LDF, 16 * wv, qtok0);
        gemm_tile_rot<CTQ, DQ>(TID_C fb, pf1b, W1, D, 128 + 16 * wv, sm.h, LDH, qtok0, wv + 1);
        store_tile<CTQ, true>(TID_C fb, bb, sm.ctx, LDF, 16 * wv, qtok0);
    } else {
        linear1<CTQ, true, DQ>(TID_C pf1a, W1, D, b1, 16 * wv, sm.h, LDH, qtok0, sm.big, LDF, 16 * wv, qtok0);
        linear1<CTQ, true, DQ>(TID_C pf1b, W1, D, b1, 128 + 16 * wv, sm.h, LDH, qtok0, sm.ctx, LDF, 16 * wv, qtok0);
    }
    const APre<DQ> pf2a = prefetch<DQ>(TID_C W2, FF, 16 * wv, 0);
    PTR(tb + 10);
    __syncthreads();
    PTR(tb + 11);
    const APre<DQ> pf2b = prefetch<DQ>(TID_C W2, FF, 16 * wv, 128);
    if (TR) {  // FFN hidden (post-ReLU): features 0-127 in big, 128-255 in ctx
        store_rows(TID_C sm.big, LDF, io.u, FF, 0, D, qtok0, b0, last, qtok1, !PSX);
        store_rows(TID_C sm.ctx, LDF, io.u, FF, D, D, qtok0, b0, last, qtok1, !PSX);
    }
    const f32x4 b24 = ln_bias(TID_C b2);
    f32x4 acc2[CTQ];
    zero(acc2);
    gemm_tile<CTQ, DQ>(TID_C acc2, pf2a, W2, FF, 16 * wv, 0, sm.big, LDF, qtok0);
    gemm_tile<CTQ, DQ>(TID_C acc2, pf2b, W2, FF, 16 * wv, 128, sm.ctx, LDF, qtok0);
    PTR(tb + 12);
    const LnPar lp2 = ln_load(TID_C b24, P + kOffs.o[layer_param(trunk, layer, N2W)], P + kOffs.o[layer_param(trunk, layer, N2B)]);
    pre_ln2();
    residual_layernorm<CTQ, TR>(TID_C sm, acc2, lp2, qtok0, LnOut{io.xhat2, PSX ? io.h2 : nullptr, io.rstd2, b0, last, !PSX});
    PTR(tb + 14);
    }
}

// ------------------------------------------------------------------ window-row projections
// Rollout fast path (uavhip_policy_forward_rows). Up to its in_proj, layer 0 of each trunk is
// token-local and linear after the embedding ReLU: Q|K|V of window row j at position s is
// Win (e_j + pos_s) + b_in = u_j + Win pos_s with u_j = Win e_j + b_in independent of s
// (transformer_net.py:57-63; post-LN encoder, so no norm in between). Consecutive rollout windows
// share 4 of their 5 rows (the observation deque, uav_env.py:241-242), so every env keeps the u
// rows of its current window in a 5-slot ring -- row r of the window sequence in slot r mod 5 --
// and the forward at sequence step g computes u for the new row only (slot g mod 5): the two
// layer-0 in_proj GEMMs shrink from 80 to 16 tokens per workgroup. Rows 0-3 of a window at step g
// are in slots (g + 1 + s) mod 5. Masked rows (all-zero padding, transformer_net.py:52-54) are
// keys masked in every layer and never reach the last token, so they read as zero.
// Ring row: actor K | V (2 x 128), then critic Q | K | V (3 x 128); Win pos_s table in front.
constexpr int kPposFloats = 2 * S * 3 * D;  // [trunk][s][384]
constexpr int kRowFloats = 5 * D;
struct RowIO {
    float* rp;  // [kPposFloats] Win pos_s, then ring [5][B][kRowFloats]
    int B, g;   // windows; sequence step of this forward
};
constexpr int kPwD = 4;  // in_proj k-blocks of the new-row GEMM loaded ahead (of 8)
template <int trunk> constexpr int row_parts() { return trunk == kActorTrunk ? 2 : 3; }  // K,V / Q,K,V
template <int NP>
struct RowPre {
    f32x4 v[2][2 * NP];  // per chunk: this thread's ring values of positions 0-3
    float pp[2][2];      // per chunk: this thread's share of the [5][192] Win pos_s rows
    f32x4 bias[3];       // in_proj bias of the wave's Q, K, V rows (new-row GEMM epilogue)
};

// Win pos_s of chunk c ([s][part * 64 + d], d < 64) -> registers; staged into sm.red (free during
// the chunk loop) by ppos_stage.
template <int trunk, int NP>
__device__ __forceinline__ void ppos_load(TID_F RowPre<NP>& r, const RowIO& rio) {
    const float* pp = rio.rp + (trunk == kActorTrunk ? 0 : S * 3 * D);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = (TIDX() + NTHR * u) % (S * 192);  // (threads past 960 reload, unused)
            const int s = i / 192, rr = i - 192 * s, part = rr >> 6, cc = rr & 63;
            r.pp[c][u] = pp[s * 3 * D + part * D + 64 * c + cc];
        }
}
template <int NP>
__device__ __forceinline__ void ppos_stage(TID_F Smem& sm, const RowPre<NP>& r, int c) {
    float* pl = reinterpret_cast<float*>(sm.red);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int i = TIDX() + NTHR * u;
        if (i < S * 192) pl[i] = r.pp[c][u];
    }
}
// Item u of chunk c for this thread: float4 q of part `part` (of the NP cached parts) of token tok
// (position tok >> 4 < 4, sample tok & 15); 16 consecutive lanes read one 256-byte row segment.
template <int NP>
__device__ __forceinline__ void ring_item(TID_F int u, int& part, int& tok) {
    const int t2 = (TIDX() >> 4) + 32 * u;
    part = t2 % NP;
    tok = t2 / NP;
}
// Chunk c of the ring rows (the critic loads chunk 1 only after its new-row GEMM: registers).
template <int trunk, int NP>
__device__ __forceinline__ void ring_load(TID_F RowPre<NP>& r, const Smem& sm, const RowIO& rio, int b0, int c) {
    constexpr int ROFF = trunk == kActorTrunk ? 0 : 2 * D;
    const float* slots = rio.rp + kPposFloats;
    const int q = TIDX() & 15;
    // predicates and offsets first (LDS reads of the mask), then the loads back to back: no LDS
    // read lands in a register of an outstanding load (that forces a vmcnt(0) drain)
    int off[2 * NP];
#pragma unroll
    for (int u = 0; u < 2 * NP; ++u) {
        int part, tok;
        ring_item<NP>(TID_C u, part, tok);
        const int s = tok >> 4, p = tok & 15, b = b0 + p;
        const bool ok = b < rio.B && !sm.mask[p * S + s];
        const int slot = (rio.g + 1 + s) % 5;
        off[u] = ok ? (slot * rio.B + b) * kRowFloats + ROFF + part * D + 64 * c + 4 * q : -1;
    }
    __builtin_amdgcn_sched_barrier(0);
    // unconditional loads (masked items read ring row 0 and are dropped): a load under a branch
    // makes the compiler's vmcnt bookkeeping assume it may be missing and wait for everything
#pragma unroll
    for (int u = 0; u < 2 * NP; ++u) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(slots + (off[u] >= 0 && !kExpHotRing ? off[u] : 4 * q));
        r.v[c][u] = off[u] >= 0 ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
}

// acc[r] += W[row[r] + i][k] . X[xtok0 + j][k] over k in [0, 128): R weight tiles against one
// activation tile (shared B operand), blocks < D from `pre` (D = KB: weights fully preloaded).
// `issued()` runs right after the last weight load is issued: loads it issues queue behind the
// GEMM's own (vmcnt retires in order), so none of the GEMM's waits cover them.
template <int R, int D, class F>
__device__ __forceinline__ void gemm_rows(TID_F f32x4 (&acc)[R], const APre<D> (&pre)[R], const float* __restrict__ W,
                                          int ldw, const int (&row)[R], const float* X, int ldx, int xtok0,
                                          F&& issued) {
    const int l = LANE(), i16 = l & 15, g = l >> 4;
    const float* xp = X + (xtok0 + i16) * ldx + 4 * g;
    f32x4 a[KB][R], b[KB];
#pragma unroll
    for (int p = 0; p < D; ++p) {
#pragma unroll
        for (int r = 0; r < R; ++r) a[p][r] = pre[r].a[p];
        b[p] = *reinterpret_cast<const f32x4*>(xp + 16 * p);
    }
#pragma unroll
    for (int i = 0; i < KB; ++i) {
        if (i + D < KB) {
#pragma unroll
            for (int r = 0; r < R; ++r)
                a[i + D][r] = *reinterpret_cast<const f32x4*>(frag_ptr(TID_C W, ldw, row[r], 0) + 256 * (i + D));
            b[i + D] = *reinterpret_cast<const f32x4*>(xp + 16 * (i + D));
        }
        if (i == (D < KB ? KB - D - 1 : 0)) issued();
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][r][j], b[i][j], acc[r], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// gemm_rows as split products: R weight tiles of a split copy against one activation tile's planes
template <int R, int D_, class F>
__device__ __forceinline__ void hgemm_rows(TID_F f32x4 (&hi)[R], f32x4 (&lo)[R], const HPre<D_> (&pre)[R],
                                           const float* __restrict__ P, int soff, int K, const int (&row)[R],
                                           const _Float16* X, int xtok0, F&& issued) {
    constexpr int NKB = D / 32;
    const int l = LANE(), i16 = l & 15, g = l >> 4;
    const _Float16* xp = X + (xtok0 + i16) * LDP + 8 * (g ^ ((i16 >> 2) & 1));  // psw's swizzle
    f16x8 a1[NKB][R], a2[NKB][R], b1[NKB], b2[NKB];
#pragma unroll
    for (int p = 0; p < D_; ++p)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            a1[p][r] = pre[r].a1[p];
            a2[p][r] = pre[r].a2[p];
        }
    b1[0] = *reinterpret_cast<const f16x8*>(xp);
    b2[0] = *reinterpret_cast<const f16x8*>(xp + kPlane);
#pragma unroll
    for (int i = 0; i < NKB; ++i) {
        if (i + 1 < NKB) {  // B one block ahead
            b1[i + 1] = *reinterpret_cast<const f16x8*>(xp + 32 * (i + 1));
            b2[i + 1] = *reinterpret_cast<const f16x8*>(xp + 32 * (i + 1) + kPlane);
        }
        if (i + D_ < NKB) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if constexpr (kExpNoWeightLoads || UAVHIP_EXP == 711) {  // timing builds only
                    a1[i + D_][r] = a1[(i + D_) % D_][r];
                    a2[i + D_][r] = a2[(i + D_) % D_][r];
                } else {
                    const f16x8* wp = hfrag_ptr(TID_C P, soff, K, row[r], 0) + 128 * (i + D_);
                    a1[i + D_][r] = wp[0];
                    a2[i + D_][r] = wp[64];
                }
            }
        }
        if (i == (D_ < NKB ? NKB - D_ - 1 : 0)) issued();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            hi[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i][r], b1[i], hi[r], 0, 0, 0);
            lo[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i][r], b2[i], lo[r], 0, 0, 0);
            lo[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[i][r], b1[i], lo[r], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}
// The new-row GEMM's weight prefetch (rows_prologue): the split copy's first blocks when layer 0's
// in_proj has one, the fp32 fragments otherwise.
template <int trunk>
constexpr bool split_ring() { return split_slot(layer_param(trunk, 0, INW)) >= 0; }
template <int trunk>
using RingPre = std::conditional_t<split_ring<trunk>(), HPre<2>, APre<kPwD>>;

// Layer 0 of a trunk on the ring: u of the new row (position 4) from `pw` (in_proj rows 128 j +
// 16 wv: this wave's Q, K and V features, all in chunk wv >> 2) and the ring rows of positions
// 0-3 from `rp`; then attention and layer_tail as in encoder_layer. Expects sm.ctx rows 64-79 =
// e of position 4 (embed_apply kEmbSplit), sm.red = Win pos_s of chunk 0 (ppos_stage).
template <int trunk, int NP>
__device__ __forceinline__ void encoder_layer_rows(TID_F Smem& sm, const float* __restrict__ P, const RingPre<trunk> (&pw)[3], RowPre<NP>& rp,
                                   const RowIO& rio, int b0) {
    constexpr bool last = trunk == kActorTrunk;  // the actor's layer 0 is its last (pruned) layer
    constexpr int P0 = 3 - NP, ROFF = trunk == kActorTrunk ? 0 : 2 * D;
    constexpr bool planes = split_tail<trunk, 0>();  // attention output as split-product planes
    [[maybe_unused]] constexpr int tb = 8 + 16 * (trunk == 0 ? 0 : 1);
    PTR(tb);
    const float* Win = P + kOffs.o[layer_param(trunk, 0, INW)];
    const int l = LANE(), i16 = l & 15, g = l >> 4, wv = TIDX() >> 6;
    const int rows[3] = {16 * wv, D + 16 * wv, 2 * D + 16 * wv};
    f32x4 acc[3] = {};
    auto ring_issue = [&] {
        ring_load<trunk>(TID_C rp, sm, rio, b0, 0);
        if (trunk == kActorTrunk) ring_load<trunk>(TID_C rp, sm, rio, b0, 1);
    };
    if constexpr (split_ring<trunk>()) {  // e of position 4 as planes in sm.ctx (embed_apply kEmbSplit)
        f32x4 lo[3] = {};
        const float inv = es_factor<trunk, 1>(sm, (S - 1) * SPW + i16);  // the new row's scale
        hgemm_rows<3, 2>(TID_C acc, lo, pw, P, split_slot(layer_param(trunk, 0, INW)), D, rows,
                         reinterpret_cast<const _Float16*>(sm.ctx), (S - 1) * SPW, ring_issue);
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[j] = (acc[j] + lo[j] * kLoScale) * inv;
    } else {
        gemm_rows<3, kPwD>(TID_C acc, pw, Win, D, rows, sm.ctx, LDH, (S - 1) * SPW, ring_issue);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[j] += rp.bias[j];  // u = Win e + b
    if (b0 + i16 < rio.B) {  // the new row -> ring slot g mod 5
        float* dst = rio.rp + kPposFloats + ((size_t)(rio.g % 5) * rio.B + b0 + i16) * kRowFloats + ROFF + 16 * wv + 4 * g;
#pragma unroll
        for (int j = P0; j < 3; ++j) *reinterpret_cast<f32x4*>(dst + (j - P0) * D) = acc[j];
    }
    if (trunk != kActorTrunk) ring_load<trunk>(TID_C rp, sm, rio, b0, 1);
    PTR(tb + 13);
    const float* pl = reinterpret_cast<const float*>(sm.red);
    const int q = TIDX() & 15;
    TailPre<trunk, 0, last, false> po;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        // Q | K | V of the chunk -> sm.big: positions 0-3 from the ring, position 4 from acc
#pragma unroll
        for (int u = 0; u < 2 * NP; ++u) {
            int part, tok;
            ring_item<NP>(TID_C u, part, tok);
            const int bp = part + P0, s = tok >> 4;
            *reinterpret_cast<f32x4*>(sm.big + tok * LDB + bp * 64 + 4 * q) =
                rp.v[c][u] + *reinterpret_cast<const f32x4*>(pl + s * 192 + bp * 64 + 4 * q);
        }
        if ((wv >> 2) == c) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int col = 64 * j + 16 * (wv & 3) + 4 * g;
                *reinterpret_cast<f32x4*>(sm.big + ((S - 1) * SPW + i16) * LDB + col) =
                    acc[j] + *reinterpret_cast<const f32x4*>(pl + (S - 1) * 192 + col);
            }
        }
        if (c == 1) po = tail_prefetch<trunk, 0, last, false>(TID_C P);
        PTR(tb + 1 + 3 * c);
        __syncthreads();
        PTR(tb + 2 + 3 * c);
        if (c == 0) ppos_stage(TID_C sm, rp, 1);  // sm.red is read again only by the chunk-1 assembly
        if (last) attention_chunk<planes, trunk, 0>(TID_C sm, c, S - 1, 1, P);
        else attention_full<planes, trunk, 0>(TID_C sm, c, P);
        __syncthreads();
        PTR(tb + 3 + 3 * c);
    }
    layer_tail<trunk, 0, last, false>(TID_C sm, P, po, TrainLayerIO{}, b0);
}

// Everything layer 0 of a trunk needs before its new-row GEMM (which then issues the ring loads
// behind its last weight loads): embedding operands, Win pos_s, the wave's in_proj weight tiles
// and bias. Ends with the embedding in sm.h / sm.ctx and Win pos_s of
// chunk 0 in sm.red, without a barrier.
template <int trunk, int NP, class H = NoHook>
__device__ __forceinline__ void rows_prologue(TID_F Smem& sm, const float* __restrict__ P, RingPre<trunk> (&pw)[3],
                                              RowPre<NP>& rp, const RowIO& rio, int b0, H hook = H{}) {
    const int wv = TIDX() >> 6;
    const EmbPre ep = embed_load<trunk>(TID_C P);
    ppos_load<trunk>(TID_C rp, rio);
    const float* Win = P + kOffs.o[layer_param(trunk, 0, INW)];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if constexpr (split_ring<trunk>()) pw[j] = hprefetch<2>(TID_C P, split_slot(layer_param(trunk, 0, INW)), D, j * D + 16 * wv, 0);
        else pw[j] = prefetch<kPwD>(TID_C Win, D, j * D + 16 * wv, 0);
    }
    const float* bin = P + kOffs.o[layer_param(trunk, 0, INB)];
#pragma unroll
    for (int j = 0; j < 3; ++j) rp.bias[j] = *reinterpret_cast<const f32x4*>(bin + j * D + 16 * wv + 4 * (LANE() >> 4));
    hook();  // behind the loads above: its latency overlaps theirs
    embed_apply<trunk, false, kEmbSplit>(TID_C sm, ep);
    ppos_stage(TID_C sm, rp, 0);
}

// 128 -> 64 (MFMA, waves 0-3) -> relu -> nout (VALU) on the last-position rows (transformer_net.py:77-91)
template <int head, int nout, int DQ = 4>
__device__ void head_mlp(TID_F Smem& sm, const float* __restrict__ P, const APre<DQ>& pw, float* out) {
    const float* W0 = P + kOffs.o[head + 0];
    const float* b0 = P + kOffs.o[head + 1];
    const float* W2 = P + kOffs.o[head + 2];
    const float* b2 = P + kOffs.o[head + 3];
    const int wv = TIDX() >> 6;
    // second layer: 16 lanes per (sample p, output a) = item p * nout + a, 4 hidden features per
    // lane; its weights and bias are loaded before the first layer's GEMM
    constexpr int kItems = SPW * nout;
    const int item = TIDX() >> 4, k4 = TIDX() & 15;
    const int p = item / nout, a = (item - p * nout) % nout;  // in range for every thread
    const f32x4 w2 = *reinterpret_cast<const f32x4*>(W2 + a * HID + 4 * k4);
    const float bb2 = b2[a];
    if (wv < HID / 16) linear1<1, true, DQ>(TID_C pw, W0, D, b0, 16 * wv, sm.h, LDH, (S - 1) * SPW, sm.z, LDZ, 16 * wv, 0);
    __syncthreads();
    if (item < kItems) {  // wave-uniform: kItems * 16 is a multiple of 64
        const f32x4 z = *reinterpret_cast<const f32x4*>(sm.z + p * LDZ + 4 * k4);
        float acc = (w2.x * z.x + w2.y * z.y) + (w2.z * z.z + w2.w * z.w);
        acc = add_xor2(add_xor1(acc));
        acc += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0x141, 0xF, 0xF, true));  // row_half_mirror
        acc += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0x140, 0xF, 0xF, true));  // row_mirror
        if (k4 == 0) out[item] = acc + bb2;
    }
    __syncthreads();
}

// Categorical(softmax(logits)) as torch.distributions evaluates it (transformer_net.py:124-144):
// p = softmax(l); p /= sum(p); lc = log(clamp(p, eps, 1 - eps)); logp = lc[a]; ent = -sum(lc * p).
struct CatVals {
    float y0, y1, s, p0, p1, c0, c1, lc0, lc1;
};
__device__ __forceinline__ CatVals categorical(float l0, float l1) {
    CatVals c;
    const float m = fmaxf(l0, l1);
    const float e0 = expf(l0 - m), e1 = expf(l1 - m);
    const float den = e0 + e1;
    c.y0 = e0 / den;
    c.y1 = e1 / den;
    c.s = c.y0 + c.y1;
    c.p0 = c.y0 / c.s;
    c.p1 = c.y1 / c.s;
    const float eps = 1.1920928955078125e-07f;
    c.c0 = fminf(fmaxf(c.p0, eps), 1.f - eps);
    c.c1 = fminf(fmaxf(c.p1, eps), 1.f - eps);
    c.lc0 = logf(c.c0);
    c.lc1 = logf(c.c1);
    return c;
}

// Training mode: relu(head.0) rows of the 16 samples (sm.z) -> z [Bm][64].
__device__ __forceinline__ void store_hidden(TID_F const Smem& sm, float* __restrict__ z, int b0) {
    if (TIDX() < SPW * HID / 4) {
        const int p = TIDX() / (HID / 4), q = TIDX() % (HID / 4);
        *reinterpret_cast<f32x4*>(z + (size_t)(b0 + p) * HID + 4 * q) =
            *reinterpret_cast<const f32x4*>(sm.z + p * LDZ + 4 * q);
    }
}

// Training mode: per-sample PPO loss terms of ppo.py:148-160 (Categorical as torch evaluates it,
// transformer_net.py:124-144) and their workgroup sums in sample order -> fpart[blk][4];
// logits / value -> smp[b][5..7] for the backward.
// One sample's four terms from its smp row o[0..4] (action, old logp, old value, return, advantage)
// and its logits / value -> t[4].
__device__ __forceinline__ void loss_terms(const float (&o)[5], float l0, float l1, float v, float eps_clip,
                                           float* t, float* verr = nullptr) {
    const CatVals c = categorical(l0, l1);
    const float logp = o[0] > 0.f ? c.lc1 : c.lc0;
    const float ratio = expf(logp - o[1]);
    const float A = o[4];
    const float s1 = ratio * A;
    const float s2 = fminf(fmaxf(ratio, 1.f - eps_clip), 1.f + eps_clip) * A;
    const float R = o[3], ov = o[2];
    const float vc = ov + fminf(fmaxf(v - ov, -eps_clip), eps_clip);
    const bool pad = o[0] < 0.f;  // padding row (idx < 0): no loss terms
    t[0] = pad ? 0.f : fminf(s1, s2);
    t[1] = pad ? 0.f : (v - R) * (v - R);
    t[2] = pad ? 0.f : (vc - R) * (vc - R);
    t[3] = pad ? 0.f : -(c.lc0 * c.p0 + c.lc1 * c.p1);
    // the largest value error itself (its square overflows fp32 from |v - R| ~ 1.8e19 on: ADVICE r05)
    if (verr) *verr = pad ? 0.f : fmaxf(fabsf(v - R), fabsf(vc - R));
}
// the block's sums in sample order (threads 0-3, one term each) -> fpart[blk][4]; thread 4: the
// block's largest value error max(|v - R|, |vc - R|) (red[4 SPW + i], loss_terms' verr) -> vpart[blk]
// (the critic backward's gradient scale, heads_bwd)
__device__ __forceinline__ void loss_block_sums(TID_F const float* red, float* fpart, float* vpart, int blk) {
    if (TIDX() < 4) {
        float acc = 0.f;
        for (int i = 0; i < SPW; ++i) acc += red[4 * i + TIDX()];
        fpart[blk * 4 + TIDX()] = acc;
    } else if (TIDX() == 4 && vpart) {
        float m = 0.f;
        for (int i = 0; i < SPW; ++i) m = fmaxf(m, red[4 * SPW + i]);
        vpart[blk] = m;
    }
}
__device__ void loss_partials(TID_F Smem& sm, const TrainIO& io, int b0) {
    float* red = sm.x;  // free after the embeddings
    if (TIDX() < SPW) {
        const int p = TIDX();
        float* o = io.smp + (size_t)(b0 + p) * 8;  // o[0..4] written by this thread at kernel start
        const float l0 = sm.logits[2 * p], l1 = sm.logits[2 * p + 1], v = sm.value[p];
        o[5] = l0;
        o[6] = l1;
        o[7] = v;
        const float oi[5] = {o[0], o[1], o[2], o[3], o[4]};
        loss_terms(oi, l0, l1, v, io.eps_clip, red + 4 * p, red + 4 * SPW + p);
    }
    __syncthreads();
    loss_block_sums(TID_C red, io.fpart, io.vpart, b0 / SPW);
}
#ifndef UAVHIP_STEPS_TU
// Trunk split: the same partials once both trunks' workgroups have written smp[5..7].
__global__ __launch_bounds__(64) void k_loss_partials(const TrainIO io) {
    __shared__ float red[5 * SPW];
    const int b0 = blockIdx.x * SPW;
    if (TIDX() < SPW) {
        const float* o = io.smp + (size_t)(b0 + TIDX()) * 8;
        const float oi[5] = {o[0], o[1], o[2], o[3], o[4]};
        loss_terms(oi, o[5], o[6], o[7], io.eps_clip, red + 4 * TIDX(), red + 4 * SPW + TIDX());
    }
    __syncthreads();
    loss_block_sums(TID_C red, io.fpart, io.vpart, blockIdx.x);
}
#endif

// The 16 windows of a workgroup -> sm.x[tok = s*16 + p][k], k padded 14 -> 16 with zeros (batch
// tail zero-filled) and the key padding mask -> sm.mask; training mode gathers minibatch row idx[b]
// of the trajectory buffer (idx < 0: a padding row, computed on row 0 and flagged by action -1 in
// smp, so it adds nothing to the loss or gradients) and, if `writer`, stores the windows, the mask
// and the per-sample loss inputs into the workspace. Ends without a barrier.
template <bool TR, bool RING = false>  // RING: only position 4's exponents are read (the new row's)
__device__ __forceinline__ void gather_windows(TID_F Smem& sm, const float* __restrict__ states, int B, const TrainIO& io,
                                               int b0, bool do_actor, const float* __restrict__ rg) {
    {   // <= 3 elements per thread, every load of a round issued before any is used: the
        // training gather is two dependent rounds (row index, then window / loss inputs)
        constexpr int kEl = (TOK * LDX + NTHR - 1) / NTHR;
        size_t src[kEl];
#pragma unroll
        for (int u = 0; u < kEl; ++u) {
            const int i = TIDX() + u * NTHR, p = (i / LDX) % SPW;
            src[u] = (size_t)(b0 + p);
            if (TR && i < TOK * LDX) src[u] = (size_t)max(io.idx[b0 + p], 0);
        }
        size_t ssrc = 0;
        [[maybe_unused]] bool pad = false;
        if (TR && TIDX() < SPW) {
            const int r = io.idx[b0 + TIDX()];
            pad = r < 0;
            ssrc = (size_t)max(r, 0);
        }
        float v[kEl];
#pragma unroll
        for (int u = 0; u < kEl; ++u) {
            const int i = TIDX() + u * NTHR;
            const int t = i / LDX, k = i - t * LDX, s = t / SPW, p = t - s * SPW;
            v[u] = (i < TOK * LDX && k < IN && b0 + p < B) ? states[(src[u] * S + s) * IN + k] : 0.f;
        }
        float ld[5];
        if (TR && TIDX() < SPW) {  // per-sample loss inputs
            ld[0] = pad ? -1.f : (float)(io.act_in[ssrc] != 0);
            ld[1] = io.oldlp_in[ssrc];
            ld[2] = io.oldv_in[ssrc];
            ld[3] = io.ret_in[ssrc];
            ld[4] = io.adv_in[ssrc];
        }
#pragma unroll
        for (int u = 0; u < kEl; ++u) {
            const int i = TIDX() + u * NTHR;
            {  // key padding mask (all-zero rows, the last never masked) from the registers: the 16
               // lanes of a token row vote; and the row's max |x_k| (layer 0's operand range)
                static_assert(LDX == 16 && NTHR % LDX == 0, "one token row = 16 lanes");
                const unsigned long long nz = __ballot(v[u] != 0.f);
                const float rmax = (UAVHIP_EXP == 62 || UAVHIP_EXP == 63) ? 0.f : row16_max(fabsf(v[u]));
                if (i < TOK * LDX && (i % LDX) == 0) {
                    const int t = i / LDX, s = t / SPW, p = t - s * SPW;
                    const bool m = (s < S - 1) && ((nz >> (LANE() & 48)) & 0xFFFFull) == 0;
                    sm.mask[p * S + s] = m;
                    sm.tmax[t] = rmax;
                    // element u's rows start at token u NTHR / LDX: the ring forward needs position 4 only
                    if (!RING || (u * NTHR) / LDX >= (S - 1) * SPW)
#pragma unroll
                    for (int ti = 0; ti < 2; ++ti)  // layer 0's constants from the table's maxima (rg)
                        sm.es[ti][t] = (signed char)range_exp(
                            e_bound_v(range_entry(rg, kRgE + 2 * ti), range_entry(rg, kRgE + 2 * ti + 1), rmax));
                    if (TR && do_actor) {
                        io.mask[(size_t)(b0 + p) * S + s] = m ? 1.f : 0.f;
                        io.tmax[(size_t)(b0 + p) * S + s] = rmax;
                    }
                }
            }
            if (i >= TOK * LDX) continue;
            sm.x[i] = v[u];
            if (TR && do_actor) io.xg[(size_t)trow(i / LDX, b0) * 16 + (i % LDX)] = v[u];
        }
        if (TR && do_actor && TIDX() < SPW) {
            float* o = io.smp + (size_t)(b0 + TIDX()) * 8;
            for (int c = 0; c < 5; ++c) o[c] = ld[c];
        }
    }
}

// The workgroup's layer-0 attention-output scale per trunk (Smem::a0f) from the max over its 80
// window rows (rows 0..TOK-1 of m, one float each): wave 0, once the rows are visible; read behind
// a later barrier. The bound holds for every sample of the workgroup. e / a0: layer 0's constants
// (policy_layout.hpp kRgE / kRgA0: Smem::rtab, or a0f_consts of the table's maxima).
// (a0f_load: wave 0's two rows per lane, issued early; a0f_finish: the reduction and the factors)
__device__ __forceinline__ float a0f_load(TID_F const float* m) {
    static_assert(TOK <= 128, "two rows per lane");
    const int l = TIDX();
    return l < 64 ? fmaxf(m[l], l + 64 < TOK ? m[l + 64] : 0.f) : 0.f;
}
// returns the workgroup's max (wave 0 only; 0 elsewhere)
__device__ __forceinline__ float a0f_finish(TID_F Smem& sm, float v, const float* e, const float* a0) {
    if (TIDX() < 64) {
        const int l = TIDX();
        v = wave_max(v);
        if (l < 2) {
            const OpSc f = a0_sc_v(e[2 * l], e[2 * l + 1], a0[2 * l], a0[2 * l + 1], v);
            sm.a0f[2 * l] = f.sc;
            sm.a0f[2 * l + 1] = f.inv;
        }
        return v;
    }
    return 0.f;
}
__device__ __forceinline__ float a0f_from_max(TID_F Smem& sm, const float* m, const float* e, const float* a0) {
    return a0f_finish(TID_C sm, a0f_load(TID_C m), e, a0);
}
__device__ __forceinline__ float a0f_from_tmax(TID_F Smem& sm) {
    if constexpr (UAVHIP_EXP != 62 && UAVHIP_EXP != 63) return a0f_from_max(TID_C sm, sm.tmax, sm.rtab + kRtE, sm.rtab + kRtA0);
    return 0.f;
}

// Fused rollout step (uavhip_rollout_step): the env step of the sampled actions (uav_env.py:295-435)
// after the forward, on the same workgroup's 16 envs.
struct EnvOut {
    int auto_reset;
    float* obs;     // [E][5][14] next windows (f32, or binary16 under UAVHIP_ENV_OBS_F16)
    double* rew;    // [E]
    uint8_t* done;  // [E]
    double* info;   // [E][UAVHIP_INFO_COUNT] (nullable)
};

// ROWS: layer 0 of both trunks on the window-row projection ring (inference only).
// ENV: the env step of the sampled actions follows (needs ROWS; envs b0 .. b0 + 15): a bit mask of
// the env-step code compiled in -- kEnvGrp (two envs per wave, N, M <= 32, both envs of every wave in
// range), kEnvWave (one env per wave, any N, M <= 64), both (chosen per wave at run time). The
// one-launch rollout instantiates one path per launch (71 -> 58.5 KB of code, 28 -> 9 VGPR spills).
enum { kEnvGrp = 1, kEnvWave = 2, kEnvBoth = 3 };
// One workgroup's whole forward (+ env step) of its 16 samples; the kernels below wrap it.
// VONLY (inference, ROWS): the critic trunk and head only -- the value of each window, nothing
// else (the rollout's bootstrap V(s_T), uavhip_policy_value_rows); the actor's ring row of the step
// is not written.
template <bool TR, bool ROWS, int ENV, bool VONLY = false>
__device__ __forceinline__ void policy_block(TID_F Smem& sm, const float* __restrict__ P, const float* __restrict__ states,
                                             int B, const int8_t* __restrict__ actions_in, uint64_t seed,
                                             uint64_t offset, const uint64_t* __restrict__ offset_dev,
                                             int8_t* __restrict__ action_out, float* __restrict__ logp_out,
                                             float* __restrict__ value_out, float* __restrict__ ent_out,
                                             float* __restrict__ logits_out, const TrainIO& io, const RowIO& rio,
                                             const uavhip_env& env, const EnvOut& eo, int bx) {
    static_assert(!(TR && ROWS), "the training forward recomputes every row");
    static_assert(!ENV || ROWS, "the fused env step follows the rollout forward");
    static_assert(!VONLY || (ROWS && !ENV && !TR), "value only: the inference ring forward");
    // training trunk split (TrainIO::split): role 1 = actor trunk + head, 2 = critic trunk + head
    // of sample block blk; role 0 = both (the rollout always)
    int blk = bx, role = VONLY ? 2 : 0;
    if constexpr (TR) {
        if (io.split) {
            role = blk < io.split ? 1 : 2;
            if (role == 2) blk -= io.split;
        }
    }
    const bool do_actor = role != 2, do_critic = role != 1;
    const int b0 = blk * SPW;
    // training forward without the trunk split (TrainIO::mix): every other group of 8 workgroups
    // runs the critic trunk first, so the two trunks' HBM-heavy activation stores and compute phases
    // overlap across the chip (as K6's BwdIO::mix)
    [[maybe_unused]] bool critic_first = false;
    if constexpr (TR) critic_first = role == 0 && io.mix && ((blk >> 3) & 1);
    PTR(0);
    // training mode: the first trunk's embedding operands and first K/V weight blocks are loaded
    // before the minibatch gather stores its rows (a load behind a store burst waits for the burst)
    [[maybe_unused]] EmbPre ep_a, ep_c;
    [[maybe_unused]] KvPre<kActorTrunk, 0, TR, kTrainSplit> pkv_a;
    [[maybe_unused]] KvPre<kCriticTrunk, 0, TR, kTrainSplit> pkv_c;
    if constexpr (TR) {
        if (do_actor && !critic_first) {
            ep_a = embed_load<kActorTrunk>(TID_C P);
            pkv_a = kv_prefetch<kActorTrunk, 0, TR, kTrainSplit>(TID_C P);
        } else {
            ep_c = embed_load<kCriticTrunk>(TID_C P);
            pkv_c = kv_prefetch<kCriticTrunk, 0, TR, kTrainSplit>(TID_C P);
        }
    }
    gather_windows<TR, ROWS>(TID_C sm, states, B, io, b0, do_actor, P + kRangeOff);
    // the sampling's Philox draws (a counter function of the sample's index alone) by the last wave's
    // first lanes while the windows load, so that the serial tail after the heads (one wave's
    // sampling) no longer runs the 10 Philox rounds (EXP=105, A/B build: drawn there)
    if constexpr (!TR && kEarlyDraw) {
        const int pd = (int)TIDX() - (NTHR - kWave);
        if (!actions_in && pd >= 0 && pd < SPW) {
            const unsigned long long c = offset + (offset_dev ? *offset_dev : 0ull) + (unsigned long long)(b0 + pd);
            const u32x4 r = philox(u32x4{(uint32_t)c, (uint32_t)(c >> 32), 0x5eedu, 0x9e37u}, (uint32_t)seed,
                                   (uint32_t)(seed >> 32));
            sm.u01[pd] = u01f(r.x);
        }
    }
    __syncthreads();
    PTR(1);
    // layer 0's attention-output scales, read behind the next barrier (the ring forward: once the
    // actor's prologue loads are issued, so that wave 0's reduction overlaps their round trip)
    if (!ROWS || !do_actor) {
        const float xm = a0f_from_tmax(TID_C sm);
        if (TR && TIDX() == 0 && io.xmax) io.xmax[blk] = xm;  // the block's range for the weight gradients
    }
    // the training forward exports its derived scales for the weight-gradient GEMM (TrainIO::rtab_out)
    if (TR && blk == 0 && TIDX() < kRtN && io.rtab_out) io.rtab_out[TIDX()] = sm.rtab[TIDX()];
    const int wv = TIDX() >> 6;
    const float* headw_a = P + kOffs.o[kActorHead];
    const float* headw_c = P + kOffs.o[kCriticHead];
    // actor trunk (1 layer) + head
    if constexpr (ROWS) {
        if (do_actor) {
            RingPre<kActorTrunk> pw[3];
            RowPre<2> rp;
            rows_prologue<kActorTrunk>(TID_C sm, P, pw, rp, rio, b0, [&] { a0f_from_tmax(TID_C sm); });
            PTR(2);
            __syncthreads();
            encoder_layer_rows<kActorTrunk>(TID_C sm, P, pw, rp, rio, b0);
        }
    }
    // training mode: the actor head's and the critic embedding's / first GEMM's operands are loaded
    // ahead of the actor's LN2 activation stores (layer_tail hook)
    // the head's weight prefetch depth: the training forward holds two blocks (four spilled one,
    // reloaded behind the activation store burst)
    constexpr int kHd = TR ? 2 : 4;
    APre<kHd> ph;
    // the training forward's actor (a lambda: TrainIO::mix calls it after the critic in half the
    // workgroups); the inference forward keeps its inline block below (the same code as before the
    // mix: as a lambda, its register allocation changed and the NOENV build of k_rollout_steps went
    // from 3 to 11 VGPR spills, skewing the env-step differential)
    [[maybe_unused]] auto actor = [&] {
        if constexpr (TR && !ROWS) {
            // the split layer-0 in_proj reads the embedding's planes in sm.ctx
            embed_apply<kActorTrunk, TR, kEmbH, split_kv<kActorTrunk, 0, TR, kTrainSplit>()>(TID_C sm, ep_a, io.e[0],
                                                                                           nullptr, b0);
            PTR(2);
            __syncthreads();
            auto hook = [&] {
                if (wv < 4) ph = prefetch<kHd>(TID_C headw_a, D, 16 * wv, 0);
                if (do_critic && !critic_first) {
                    ep_c = embed_load<kCriticTrunk>(TID_C P);
                    pkv_c = kv_prefetch<kCriticTrunk, 0, TR, kTrainSplit>(TID_C P);
                }
            };
            encoder_layer<kActorTrunk, 0, true, TR, decltype(hook), kTrainSplit>(TID_C sm, P, pkv_a, io.L[0], b0, hook);
            __syncthreads();
            PTR(3);
            head_mlp<kActorHead, 2, kHd>(TID_C sm, P, ph, sm.logits);
            store_hidden(TID_C sm, io.z[0], b0);  // before the critic's LayerNorm partials reuse sm.z
        }
    };
    if constexpr (TR) {
        if (do_actor && !critic_first) actor();
    } else if (do_actor) {
        if constexpr (!ROWS) {
            APre<2> pkv = prefetch<2>(TID_C P + kOffs.o[layer_param(kActorTrunk, 0, INW)], D, kv_row(wv, 0), 0);
            embed<kActorTrunk, TR>(TID_C sm, P, io.e[0], nullptr, b0);
            PTR(2);
            __syncthreads();
            encoder_layer<kActorTrunk, 0, true, TR>(TID_C sm, P, pkv, io.L[0], b0);
        }
        if (wv < 4) ph = prefetch<kHd>(TID_C headw_a, D, 16 * wv, 0);
        __syncthreads();
        PTR(3);
        head_mlp<kActorHead, 2, kHd>(TID_C sm, P, ph, sm.logits);
    }  // do_actor
    PTR(4);
    // fused env step (ENV): two envs per wave side by side, state loads issued before the critic head
    [[maybe_unused]] const bool env_grp =
        (ENV & kEnvGrp) && env.N <= envgrp::L && env.M <= envgrp::L && b0 + 2 * wv + 1 < B;
    [[maybe_unused]] envgrp::GRegs gR;
    [[maybe_unused]] envgrp::GPending gq;
    if (do_critic) {
        // critic trunk (2 layers) + head
        if constexpr (ROWS) {
            RingPre<kCriticTrunk> pw[3];
            RowPre<3> rp;
            rows_prologue<kCriticTrunk>(TID_C sm, P, pw, rp, rio, b0);
            __syncthreads();
            encoder_layer_rows<kCriticTrunk>(TID_C sm, P, pw, rp, rio, b0);
        }
        KvPre<kCriticTrunk, 1, TR, TR ? kTrainSplit : true> pkv;
        if constexpr (!ROWS) {
            if constexpr (TR) {
                embed_apply<kCriticTrunk, TR, kEmbH, split_kv<kCriticTrunk, 0, TR, kTrainSplit>()>(TID_C sm, ep_c, io.e[1],
                                                                                                 nullptr, b0);
                __syncthreads();
                auto hook = [&] { pkv = kv_prefetch<kCriticTrunk, 1, TR, kTrainSplit>(TID_C P); };
                encoder_layer<kCriticTrunk, 0, false, TR, decltype(hook), kTrainSplit>(TID_C sm, P, pkv_c, io.L[1], b0, hook);
            } else {
                APre<2> pkv0 = prefetch<2>(TID_C P + kOffs.o[layer_param(kCriticTrunk, 0, INW)], D, kv_row(wv, 0), 0);
                embed<kCriticTrunk, TR>(TID_C sm, P, io.e[1], nullptr, b0);
                __syncthreads();
                encoder_layer<kCriticTrunk, 0, false, TR>(TID_C sm, P, pkv0, io.L[1], b0);
            }
        }
        if constexpr (!TR) pkv = kv_prefetch<kCriticTrunk, 1, TR>(TID_C P);
        __syncthreads();
        if constexpr (TR) {
            auto hook = [&] {
                if (wv < 4) ph = prefetch<kHd>(TID_C headw_c, D, 16 * wv, 0);
            };
            encoder_layer<kCriticTrunk, 1, true, TR, decltype(hook), kTrainSplit>(TID_C sm, P, pkv, io.L[2], b0, hook);
        } else {
            encoder_layer<kCriticTrunk, 1, true, TR>(TID_C sm, P, pkv, io.L[2], b0);
        }
        // the env step's state loads land while the critic head runs
        if constexpr ((ENV & kEnvGrp) && !kExpNoEnv) {
            if (env_grp) {
                const int le = tid_env() & 63;
                envgrp::gload_issue(gR, gq, env, b0 + 2 * (int)(tid_env() >> 6) + (le >> 5), le & 31);
            }
        }
        if (!TR && wv < 4) ph = prefetch<kHd>(TID_C headw_c, D, 16 * wv, 0);
        __syncthreads();
        PTR(5);
        head_mlp<kCriticHead, 1, kHd>(TID_C sm, P, ph, sm.value);
        PTR(6);
        if (TR) store_hidden(TID_C sm, io.z[1], b0);
    }  // do_critic
    if constexpr (TR) {
        if (critic_first) {  // the actor's operands now (not prefetched: the critic's hooks are full)
            ep_a = embed_load<kActorTrunk>(TID_C P);
            pkv_a = kv_prefetch<kActorTrunk, 0, TR, kTrainSplit>(TID_C P);
            __syncthreads();  // the actor's trunk reuses the critic's buffers (sm.z after store_hidden)
            actor();
        }
    }
    if (TR) {
        if (role == 0) {
            loss_partials(TID_C sm, io, b0);
        } else if (TIDX() < SPW) {  // trunk split: this trunk's head outputs -> smp[5..7]
            float* o = io.smp + (size_t)(b0 + TIDX()) * 8;
            if (do_actor) {
                o[5] = sm.logits[2 * TIDX()];
                o[6] = sm.logits[2 * TIDX() + 1];
            } else {
                o[7] = sm.value[TIDX()];
            }
        }
        return;
    }
    if constexpr (VONLY) {  // the value alone
        if (TIDX() < SPW && b0 + (int)TIDX() < B) value_out[b0 + TIDX()] = sm.value[TIDX()];
        return;
    }
    // Categorical(softmax(logits)): sample / log_prob / entropy (transformer_net.py:118-122)
    if (TIDX() < SPW) {
        const int p = TIDX(), b = b0 + p;
        if (b < B) {
            const float l0 = sm.logits[2 * p], l1 = sm.logits[2 * p + 1];
            const float m = fmaxf(l0, l1);
            const float lse = m + logf(expf(l0 - m) + expf(l1 - m));
            const float lp0 = l0 - lse, lp1 = l1 - lse;
            const float p0 = expf(lp0), p1 = expf(lp1);
            int a;
            if (actions_in) {
                a = actions_in[b] != 0;
            } else {
                float u;
                if constexpr (kEarlyDraw) {
                    u = sm.u01[p];
                } else {
                    const unsigned long long c = offset + (offset_dev ? *offset_dev : 0ull) + (unsigned long long)b;
                    const u32x4 r = philox(u32x4{(uint32_t)c, (uint32_t)(c >> 32), 0x5eedu, 0x9e37u}, (uint32_t)seed,
                                           (uint32_t)(seed >> 32));
                    u = u01f(r.x);
                }
                a = u < p0 ? 0 : 1;
            }
            if (action_out) action_out[b] = (int8_t)a;
            if (logp_out) logp_out[b] = a ? lp1 : lp0;
            if (ent_out) ent_out[b] = -(p0 * lp0 + p1 * lp1);
            if (value_out) value_out[b] = sm.value[p];
            if (logits_out) { logits_out[2 * b] = l0; logits_out[2 * b + 1] = l1; }
            if (ENV) sm.mask[p] = a;  // the key mask is dead after the forward
        }
    }
    PTR(7);
    if constexpr (ENV && kExpNoEnv) {  // NOENV: the next windows without the env step (timing only)
        __syncthreads();
        for (int i = TIDX(); i < SPW * envdev::kObs; i += NTHR) {
            const int p = i / envdev::kObs, r = i - p * envdev::kObs, s_ = r / IN, k = r - s_ * IN;
            const int e = b0 + p;
            const float v = sm.x[((s_ < S - 1 ? s_ + 1 : S - 1) * SPW + p) * LDX + k];
            if (e < B) envdev::obs_at(eo.obs, e, false)[r] = k == IN - 1 ? 1.0f : v;
        }
    }
    if constexpr (ENV && !kExpNoEnv) {
        // UAVEnv.step of this workgroup's 16 envs, two per wave (one env per wave at a time,
        // envdev::step_once on register state; the wave's row scratch in the dead sm.x). Both envs'
        // registers are loaded in one round before either steps.
        __syncthreads();
        PTR(60);
        using namespace envdev;
        const int lane = tid_env() & 63, wve = tid_env() >> 6, e0 = b0 + 2 * wve;
        if constexpr ((ENV & kEnvGrp) != 0) if (env_grp) {
            // both envs side by side, 32 lanes each (env_group.hpp); window scratch in the dead sm.h
            const int j = lane & 31, g = lane >> 5, e = e0 + g;
            envgrp::GRegs& R = gR;
            R.tab = nullptr;
            R.win = sm.h + (2 * wve + g) * envgrp::kWin;
            envgrp::gload_finish(R, gq, env, e, j);
            PTR(61);
            envgrp::gstep<false>(R, env, e, j, sm.mask[2 * wve + g], eo.auto_reset, obs_at(eo.obs, e, obs_f16(env)),
                          eo.rew + e, eo.done + e, eo.info ? eo.info + (size_t)e * UAVHIP_INFO_COUNT : nullptr);
            PTR(62);
            if constexpr (UAVHIP_EXP == 42) envgrp::gstore_regs(R, env, e, j);  // timing build: every entry
            else envgrp::gstore_delta(R, env, e, j);  // only the entries the step changed
            PTR(63);
        }
        if constexpr ((ENV & kEnvWave) != 0) if (!env_grp && e0 < B) {
            const bool two = e0 + 1 < B;
            EnvRegs<1> R0, R1;
            R0.row = R1.row = sm.x + 16 * wve;
            load_regs<1, true>(R0, env, e0, lane);
            if (two) load_regs<1, true>(R1, env, e0 + 1, lane);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (k == 1 && !two) break;
                EnvRegs<1>& R = k ? R1 : R0;
                const int e = e0 + k;
                step_once<1, false>(R, env, e, lane, sm.mask[2 * wve + k], eo.auto_reset,
                                    obs_at(eo.obs, e, obs_f16(env)), eo.rew + e, eo.done + e,
                                    eo.info ? eo.info + (size_t)e * UAVHIP_INFO_COUNT : nullptr);
                store_regs(R, env, e, lane);
            }
        }
    }
}

template <bool TR, bool ROWS = false, int ENV = 0, bool VONLY = false>
__global__ __launch_bounds__(NTHR) void k_policy_forward(const float* __restrict__ P, const float* __restrict__ states,
                                                         int B, const int8_t* __restrict__ actions_in, uint64_t seed,
                                                         uint64_t offset, const uint64_t* __restrict__ offset_dev,
                                                         int8_t* __restrict__ action_out,
                                                         float* __restrict__ logp_out, float* __restrict__ value_out,
                                                         float* __restrict__ ent_out, float* __restrict__ logits_out,
                                                         const TrainIO io, const RowIO rio, const uavhip_env env,
                                                         const EnvOut eo) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    // the younger half (waves 4-7, the arbitration loser of every phase) at priority 1
    if (tid_x() >= NTHR / 2) __builtin_amdgcn_s_setprio(1);
    load_rtab(TID_K sm, P);
    policy_block<TR, ROWS, ENV, VONLY>(TID_K sm, P, states, B, actions_in, seed, offset, offset_dev, action_out, logp_out,
                                       value_out, ent_out, logits_out, io, rio, env, eo, blockIdx.x);
}

// Multi-step fused rollout (uavhip_rollout_steps). A workgroup's 16 envs and their windows, ring
// rows and env state are touched by no other workgroup, so one launch runs n consecutive steps of
// them with only a workgroup barrier in between (the step's global stores -- next windows, ring
// row, env state -- are read by the next step's waves of the same workgroup: __syncthreads orders
// them, workgroup scope). Step t: windows obs[t] -> actions / logp / value [t], obs[t + 1],
// reward / done / info [t]; ring step g + t; sampling counters offset + t * off_stride + b. Saves
// the per-launch tail (the slowest of 256 workgroups, +2.6 % over the median) and start-up.
struct StepSeq {
    int n;                 // steps in this launch
    long long obs_stride;  // floats from obs[t] to obs[t + 1] (E * 5 * 14)
    uint64_t off_stride;   // sampling counter advance per step
};
// k_rollout_steps is compiled in its own translation unit (rollout_steps.hip: this file with
// UAVHIP_STEPS_TU + UAVHIP_TID_LAUNDER); uavhip_rollout_steps launches it through this.
int launch_rollout_steps(const float* P, float* obs, int B, uint64_t seed, uint64_t offset,
                         const uint64_t* offset_dev, int8_t* actions, float* logp, float* value, const RowIO& rio,
                         const uavhip_env& env, const EnvOut& eo, const StepSeq& seq, hipStream_t stream);
#ifdef UAVHIP_STEPS_TU
// All of the launch's arguments in one struct: the kernel's only parameter, so the kernarg
// segment holds exactly this struct at offset 0.
struct StepsArgs {
    const float* P;
    const float* states;
    int B;
    uint64_t seed, offset;
    const uint64_t* offset_dev;
    int8_t* action_out;
    float *logp_out, *value_out;
    RowIO rio;
    uavhip_env env;
    EnvOut eo;
    StepSeq seq;
};
template <int ENVP>  // kEnvGrp / kEnvWave (launch_rollout_steps picks)
__global__ __launch_bounds__(NTHR) void k_rollout_steps(const StepsArgs args) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    if (threadIdx.x >= NTHR / 2) __builtin_amdgcn_s_setprio(1);
    if (threadIdx.x == 0) g_tid_zero = 0;
    load_rtab(TID_K sm, args.P);  // the weights are the launch's: once
    for (int t = 0; t < args.seq.n; ++t) {
        __syncthreads();  // g_tid_zero; the previous step's LDS scratch and global stores
        // Every argument is read through a kernarg pointer laundered per step, so the loads sit where
        // the body uses them instead of being hoisted out of the loop and kept live (spilled) across
        // the whole body; pointers loaded from the constant address space are still known global.
        typedef const __attribute__((address_space(4))) StepsArgs* kargs;
        kargs ka = (kargs)__builtin_amdgcn_kernarg_segment_ptr();
        int bx = blockIdx.x;
        unsigned tid = threadIdx.x;  // the forward helpers' lane index, opaque per step (TID_F)
        asm volatile("" : "+s"(ka), "+s"(bx), "+v"(tid));
        tid &= NTHR - 1;  // threadIdx.x's range, which the launder hides from the compiler
        const StepsArgs& a = *(const StepsArgs*)ka;
        const size_t o = (size_t)t * a.B;
        const RowIO r{a.rio.rp, a.rio.B, a.rio.g + t};
        const EnvOut e{a.eo.auto_reset, a.eo.obs + t * a.seq.obs_stride, a.eo.rew + o, a.eo.done + o,
                       a.eo.info ? a.eo.info + o * UAVHIP_INFO_COUNT : nullptr};
        policy_block<false, true, ENVP>(tid, sm, a.P, a.states + t * a.seq.obs_stride, a.B, nullptr, a.seed,
                                        a.offset + t * a.seq.off_stride, a.offset_dev, a.action_out + o, a.logp_out + o,
                                        a.value_out + o, nullptr, nullptr, TrainIO{}, r, a.env, e, bx);
    }
}
#ifdef UAVHIP_POLICY_TRACE
extern "C" int uavhip_steps_trace(unsigned long long* out, int n) {  // the last step's k_rollout_steps stamps
    const int total = 256 * 2 * kTraceSlots;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ptrace), sizeof(unsigned long long) * (n < total ? n : total), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
int launch_rollout_steps(const float* P, float* obs, int B, uint64_t seed, uint64_t offset,
                         const uint64_t* offset_dev, int8_t* actions, float* logp, float* value, const RowIO& rio,
                         const uavhip_env& env, const EnvOut& eo, const StepSeq& seq, hipStream_t stream) {
    // two envs per wave wherever every wave's envs come in pairs (policy_block's env_grp for all of
    // them): the grouped path alone; else the one-env-per-wave path alone (bitwise the same steps)
    const StepsArgs sa{P, obs, B, seed, offset, offset_dev, actions, logp, value, rio, env, eo, seq};
    if (env.N <= envgrp::L && env.M <= envgrp::L && B % 2 == 0)
        hipLaunchKernelGGL(k_rollout_steps<kEnvGrp>, dim3((B + SPW - 1) / SPW), dim3(NTHR), 0, stream, sa);
    else
        hipLaunchKernelGGL(k_rollout_steps<kEnvWave>, dim3((B + SPW - 1) / SPW), dim3(NTHR), 0, stream, sa);
    return check_launch("k_rollout_steps");
}
#endif  // UAVHIP_STEPS_TU

#ifndef UAVHIP_STEPS_TU
// Ring fill of one trunk: u rows of positions 0-3 of the workgroup's 16 windows -> slots
// (g + 1 + s) mod 5, the same GEMM (k order, bias add) as the forward's new-row u. Every global
// operand of a trunk's fill -- the embedding's, the wave's in_proj row tiles (all k blocks) and
// their biases -- is one FillPre, loaded ahead (k_policy_rows_fill: the actor's before the window
// rows, the critic's before the actor's GEMMs), so a trunk's fill waits for one L2 round trip
// instead of one per row tile and k-block pair.
template <int trunk>
struct FillPre {
    static constexpr int NP = row_parts<trunk>();
    using W = std::conditional_t<split_ring<trunk>(), HPre<4>, APre<KB>>;
    EmbPre ep;
    W w[NP];
    f32x4 bb[NP];
};
template <int trunk>
__device__ __forceinline__ void fill_load_w(FillPre<trunk>& r, const float* __restrict__ P) {
    constexpr int NP = row_parts<trunk>(), P0 = 3 - NP;
    const int g = lane_id() >> 4, wv = tid_x() >> 6;
    const float* bin = P + kOffs.o[layer_param(trunk, 0, INB)];
#pragma unroll
    for (int j = P0; j < 3; ++j) {
        const int row = j * D + 16 * wv;
        if constexpr (split_ring<trunk>()) r.w[j - P0] = hprefetch<4>(P, split_slot(layer_param(trunk, 0, INW)), D, row, 0);
        else r.w[j - P0] = prefetch<KB>(P + kOffs.o[layer_param(trunk, 0, INW)], D, row, 0);
        r.bb[j - P0] = *reinterpret_cast<const f32x4*>(bin + row + 4 * g);
    }
}
// `after_first` runs after the first row tile's GEMM (the next trunk's weights are issued there,
// once this trunk's first tile has released its registers).
template <int trunk, class F>
__device__ void rows_fill_trunk(Smem& sm, const float* __restrict__ P, const FillPre<trunk>& pre, const RowIO& rio,
                                int b0, F after_first) {
    constexpr int NP = row_parts<trunk>(), P0 = 3 - NP, ROFF = trunk == kActorTrunk ? 0 : 2 * D;
    const float* Win = P + kOffs.o[layer_param(trunk, 0, INW)];
    const int l = lane_id(), i16 = l & 15, g = l >> 4, wv = tid_x() >> 6;
    embed_apply<trunk, false, kEmbRows>(sm, pre.ep);
    __syncthreads();
    float* slots = rio.rp + kPposFloats;
#pragma unroll
    for (int j = P0; j < 3; ++j) {
        const int row = j * D + 16 * wv;
        f32x4 acc[S - 1];
        zero(acc);
        if constexpr (split_ring<trunk>()) {  // the forward's new-row GEMM as split products: the same sums
            constexpr int si = split_slot(layer_param(trunk, 0, INW));
            f32x4 lo[S - 1];
            zero(lo);
            hgemm_tile<S - 1, 4>(acc, lo, pre.w[j - P0], P, si, D, row, 0, reinterpret_cast<const _Float16*>(sm.ctx), 0);
#pragma unroll
            for (int s = 0; s < S - 1; ++s) acc[s] = (acc[s] + lo[s] * kLoScale) * es_factor<trunk, 1>(sm, s * SPW + i16);
        } else {
            gemm_tile<S - 1, KB>(acc, pre.w[j - P0], Win, D, row, 0, sm.ctx, LDH, 0);
        }
        if (j == P0) after_first();
        const f32x4 bb = pre.bb[j - P0];
        const int b = b0 + i16;
        if (b < rio.B) {
#pragma unroll
            for (int s = 0; s < S - 1; ++s)
                *reinterpret_cast<f32x4*>(slots + ((size_t)((rio.g + 1 + s) % 5) * rio.B + b) * kRowFloats + ROFF +
                                          (j - P0) * D + 16 * wv + 4 * g) = acc[s] + bb;
        }
    }
    __syncthreads();  // sm.ctx is the next trunk's embedding
}

// Win pos_s of one trunk -> rp[trunk][s][384] (no bias): pos rows as activation tile columns 0-4;
// part j = rows [128 j, 128 j + 128) (Q, K or V), its weight blocks loaded before the pos rows.
constexpr int kPposParts = 6;  // (trunk, j) pairs
template <int trunk>
__device__ void rows_ppos_part(Smem& sm, const float* __restrict__ P, float* out, int j) {
    const float* Win = P + kOffs.o[layer_param(trunk, 0, INW)];
    const float* pos = P + kOffs.o[trunk + POS];
    const int l = lane_id(), i16 = l & 15, g = l >> 4, wv = tid_x() >> 6;
    const int row = j * D + 16 * wv;
    const APre<KB> pw = prefetch<KB>(Win, D, row, 0);
    for (int i = tid_x(); i < SPW * D; i += NTHR) {
        const int t = i / D, k = i - t * D;
        sm.h[t * LDH + k] = t < S ? pos[t * D + k] : 0.f;
    }
    __syncthreads();
    f32x4 acc[1];
    zero(acc);
    gemm_tile<1, KB>(acc, pw, Win, D, row, 0, sm.h, LDH, 0);
    if (i16 < S) *reinterpret_cast<f32x4*>(out + i16 * 3 * D + row + 4 * g) = acc[0];
}

// uavhip_policy_forward_rows with fill: rebuilds the ring rows of positions 0-3 of every window
// (blocks < nb) and the Win pos_s table (blocks < kPposParts, one (trunk, part) each, after their
// fill: the grid is max(nb, kPposParts) blocks). The table used to be one extra block of its own:
// with one workgroup per CU it waited for a free CU and then ran six serial GEMMs, 28 us per
// launch against ~10 us now (r04x / r04y).
__global__ __launch_bounds__(NTHR) void k_policy_rows_fill(const float* __restrict__ P,
                                                           const float* __restrict__ states, const RowIO rio) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    const int nb = (rio.B + SPW - 1) / SPW;
    load_rtab(sm, P);
    if ((int)blockIdx.x < nb) {
        const int b0 = blockIdx.x * SPW;
        FillPre<kActorTrunk> fa;
        FillPre<kCriticTrunk> fc;
        fa.ep = embed_load<kActorTrunk>(P);
        fill_load_w(fa, P);
        fc.ep = embed_load<kCriticTrunk>(P);
        for (int i = tid_x(); i < (S - 1) * SPW * LDX; i += NTHR) {  // positions 0-3 only
            const int t = i / LDX, k = i - t * LDX, s = t / SPW, p = t - s * SPW;
            const float x = (k < IN && b0 + p < rio.B) ? states[((size_t)(b0 + p) * S + s) * IN + k] : 0.f;
            sm.x[i] = x;
            const float rmax = row16_max(fabsf(x));  // the row's range (one 16-lane row per token)
            if (k == 0) {
                sm.tmax[t] = rmax;
#pragma unroll
                for (int ti = 0; ti < 2; ++ti)  // as gather_windows
                    sm.es[ti][t] = (signed char)range_exp(
                        e_bound_v(range_entry(P + kRangeOff, kRgE + 2 * ti), range_entry(P + kRangeOff, kRgE + 2 * ti + 1),
                                  rmax));
            }
        }
        __syncthreads();
        rows_fill_trunk<kActorTrunk>(sm, P, fa, rio, b0, [&] { fill_load_w(fc, P); });
        rows_fill_trunk<kCriticTrunk>(sm, P, fc, rio, b0, [] {});  // ends with a barrier
    }
    if ((int)blockIdx.x < kPposParts) {  // block-uniform
        const int t = blockIdx.x;
        if (t < 3) rows_ppos_part<kActorTrunk>(sm, P, rio.rp, t);
        else rows_ppos_part<kCriticTrunk>(sm, P, rio.rp + S * 3 * D, t - 3);
    }
}

// ================================================================== K6: fused training backward
// Mirror of the forward for one 16-sample workgroup: gradients flow through the LDS-resident
// [tok][feature] rows, the dX GEMMs run transposed on the MFMA with the transposed weights
// (policy_pack_transposed) as A operands, and only the dY operands of the weight-gradient GEMMs
// (df, du, dz1, dqkv) plus per-workgroup LayerNorm / embedding partials go to HBM.
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ float add_ror4(float v) {  // row_ror:4 inside each row of 16 lanes
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, true));
}
__device__ __forceinline__ float add_ror8(float v) {
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, true));
}
__device__ __forceinline__ float row16_sum(float v) { return add_ror8(add_ror4(add_xor2(add_xor1(v)))); }
__device__ __forceinline__ float hsum(f32x4 v) { return (v.x + v.y) + (v.z + v.w); }

// LayerNorm backward (torch's formula) on LDS rows, tokens [t0, TOK), 16 lanes per token and 8
// features per lane: g = src * w; dz = rstd * (g - mean(g) - xhat * mean(g * xhat)) -> dst (LDS)
// and gout (workspace rows). Workgroup partials, reduced over the 32 lane groups through `scratch`
// (12 KiB floats): dw = sum src * xhat, db = sum src -> part[0..127], [128..255]; the bias
// gradient of the linear that produced the LayerNorm input, sum dz -> bias[0..127]. Ends without a
// barrier after the partials are written (scratch is read until then).
// Its global operands -- the weight and this lane group's (<= 3) tokens' xhat rows and 1/std -- in
// one round trip, issued by the caller ahead of time (ln_bwd_load) so the HBM latency hides under
// the preceding phase.
constexpr int kLnIt = (TOK + NTHR / 16 - 1) / (NTHR / 16);
struct LnBwdPre {
    f32x4 w0, w1, X0[kLnIt], X1[kLnIt];
    float RS[kLnIt];
};
__device__ __forceinline__ void ln_bwd_load(LnBwdPre& a, const float* __restrict__ xhat, const float* __restrict__ rstd,
                                            const float* __restrict__ w, int t0, int b0, bool compact, int t1 = TOK) {
    const int f0 = 8 * (tid_x() & 15), grp = tid_x() >> 4;
    a.w0 = ld4(w + f0);
    a.w1 = ld4(w + f0 + 4);
#pragma unroll
    for (int it = 0; it < kLnIt; ++it) {
        const int tok = t0 + grp + it * (NTHR / 16);
        if (tok < t1) {  // wave-uniform
            const size_t r = (size_t)orow(tok, b0, compact);
            a.X0[it] = ld4(xhat + r * D + f0);
            a.X1[it] = ld4(xhat + r * D + f0 + 4);
            a.RS[it] = rstd[r];
        }
    }
}
// PL: dst receives the two fp16 planes of the split products (the next GEMM's operand) instead of fp32.
template <bool PL = false>
__device__ void ln_bwd_lds(const float* src, float* dst, const LnBwdPre& a, float* __restrict__ gout,
                           float* __restrict__ part, float* __restrict__ bias, int t0, int b0, bool compact,
                           float* scratch, int t1 = TOK) {
    const int j = tid_x() & 15, grp = tid_x() >> 4;
    const int f0 = 8 * j;
    const f32x4 w0 = a.w0, w1 = a.w1;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    f32x4 pw0 = zero4, pw1 = zero4, pb0 = zero4, pb1 = zero4, pd0 = zero4, pd1 = zero4;
    constexpr int kIt = kLnIt;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        const int tok = t0 + grp + it * (NTHR / 16);
        if (tok >= t1) continue;
        const size_t r = (size_t)orow(tok, b0, compact);
        const f32x4 g0 = ld4(src + tok * LDH + f0), g1 = ld4(src + tok * LDH + f0 + 4);
        const f32x4 x0 = a.X0[it], x1 = a.X1[it];
        const float rs = a.RS[it];
        const f32x4 gw0 = g0 * w0, gw1 = g1 * w1;
        const float m1 = row16_sum(hsum(gw0) + hsum(gw1)) * (1.0f / D);
        const float m2 = row16_sum(hsum(gw0 * x0) + hsum(gw1 * x1)) * (1.0f / D);
        const f32x4 d0 = rs * (gw0 - m1 - x0 * m2), d1 = rs * (gw1 - m1 - x1 * m2);
        if constexpr (PL) {
            hsplit_store(reinterpret_cast<_Float16*>(dst), psw(tok, f0), d0);
            hsplit_store(reinterpret_cast<_Float16*>(dst), psw(tok, f0 + 4), d1);
        } else {
            st4(dst + tok * LDH + f0, d0);
            st4(dst + tok * LDH + f0 + 4, d1);
        }
        dy_st4(gout + r * D + f0, d0);
        dy_st4(gout + r * D + f0 + 4, d1);
        pw0 += g0 * x0; pw1 += g1 * x1;
        pb0 += g0; pb1 += g1;
        pd0 += d0; pd1 += d1;
    }
    float* sc = scratch + grp * 3 * D;
    st4(sc + f0, pw0); st4(sc + f0 + 4, pw1);
    st4(sc + D + f0, pb0); st4(sc + D + f0 + 4, pb1);
    st4(sc + 2 * D + f0, pd0); st4(sc + 2 * D + f0 + 4, pd1);
    __syncthreads();
    if (tid_x() < 3 * D) {
        float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < NTHR / 16; ++q) s4[q & 3] += scratch[q * 3 * D + tid_x()];
        const float tot = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        if (tid_x() < 2 * D) part[tid_x()] = tot;
        else bias[tid_x() - 2 * D] = tot;
    }
}

// Attention backward for heads [4c, 4c+4), P recomputed from q, k (from the workspace qkv rows);
// with g = d(attention output) of the query rows (sm.ctx):
//   dv_j = sum_i P_ij g_i; dP_ij = g_i . v_j; dS_ij = P_ij (dP_ij - sum_k P_ik dP_ik);
//   dq_i = sum_j dS_ij k_j / 4; dk_j = sum_i dS_ij q_i / 4.
// One (sample, head) task per 8 lanes, 2 of the 16 head dims each (all 512 threads; dot products
// reduced over the 8 lanes with two quad permutes and a half-row mirror). dq | dk | dv ->
// sm.big [tok][3 x 64] (the forward's chunk layout; pruned layers: dq zero outside the token-4
// query rows); the caller copies them to the dqkv rows. Per-wave sums over the wave's 2 samples of
// dq, dk, dv -> scratch [wave][192] (in_proj bias partials).
__device__ __forceinline__ float add_hmirror8(float v) {  // + lane 7 - i within each group of 8
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true));
}
__device__ __forceinline__ float sum8(float v) { return add_hmirror8(add_xor2(add_xor1(v))); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 ld2(const float* p) { return *reinterpret_cast<const f32x2*>(p); }
// K6 reads the forward's Q | K | V rows (read once, by K6 alone) with non-temporal loads: they do not
// displace the L2 lines the rest of the backward re-reads (same-box, three pairs at minibatch 4096:
// K6 106.7 -> 102.1 us on average, profiles/r06s_train_ab_nt_qkv_loads.txt). EXP=87 (A/B build): plain.
__device__ __forceinline__ f32x2 ld2_once(const float* p) {
    if constexpr (UAVHIP_EXP != 87) return __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(p));
    else return ld2(p);
}
__device__ __forceinline__ void st2(float* p, f32x2 v) { *reinterpret_cast<f32x2*>(p) = v; }

// The chunk's saved Q / K / V values of this thread (2 head dims of one (sample, head)), loaded by
// the caller well ahead of attn_bwd_chunk: the rows come from HBM (written by the forward long before).
struct AttnPre {
    f32x2 k[S], v[S], q[S];
};
// qsel >= 0 (position split): the one query position qsel; else every position (full layer) or
// position 4 (pruned layer)
template <bool last>
__device__ __forceinline__ void attn_bwd_load(AttnPre& a, const float* __restrict__ qkv, int c, int b0, int qsel = -1) {
    const int o8 = tid_x() & 7, hh = (tid_x() >> 3) & 3, p = tid_x() >> 5;
    const int col = 64 * c + hh * HD + 2 * o8;
    const size_t rb = kExpNoQkvStream ? (size_t)p * S : (size_t)(b0 + p) * S;
#pragma unroll
    for (int j = 0; j < S; ++j) {
        a.k[j] = ld2_once(qkv + (rb + j) * 3 * D + D + col);
        a.v[j] = ld2_once(qkv + (rb + j) * 3 * D + 2 * D + col);
    }
#pragma unroll
    for (int i = 0; i < S; ++i)
        if (qsel >= 0 ? i == qsel : (!last || i == S - 1)) a.q[i] = ld2_once(qkv + (rb + i) * 3 * D + col);
}
// SP (split-product backward): dq | dk | dv go to sm.big as the two fp16 planes of the W_in^T GEMM's
// operand -- both planes of a token in one row, [tok][plane 1: 192 halves | plane 2: 192 | pad 16]
// (800-B rows: token i16 at bank offset 8 i16, conflict-free ds_read_b128 operand reads) -- and,
// exact, straight to the dqkv rows (dqkv != nullptr).
constexpr int kLdbP = 2 * LDB, kPlaneB = 3 * 64;  // halves per row, plane 2 within the row
static_assert(kPlaneB + 3 * 64 <= kLdbP, "both planes in an LDB row");
__device__ __forceinline__ void attn_out2(Smem& sm, float* __restrict__ dqkv, int b0, int tok, int col, int part,
                                          int c, f32x2 v, bool sp, float* __restrict__ kvc = nullptr, int kblk = 0) {
    if (sp) {
        _Float16* bp = reinterpret_cast<_Float16*>(sm.big) + tok * kLdbP + part * 64 + col;
        const _Float16 a0 = (_Float16)v.x, a1 = (_Float16)v.y;
        typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<f16x2*>(bp) = f16x2{a0, a1};
        *reinterpret_cast<f16x2*>(bp + kPlaneB) = f16x2{f16_lo(v.x, a0), f16_lo(v.y, a1)};
        if (kvc && part > 0)  // position split: this query position's share of every position's dk / dv
            st2(kvc + ((size_t)kblk * TOK + tok) * 2 * D + (part - 1) * D + 64 * c + col, v);
        else
            dy_st2(dqkv + (size_t)trow(tok, b0) * 3 * D + part * D + 64 * c + col, v);
    } else {
        st2(sm.big + tok * LDB + part * 64 + col, v);
    }
}
template <bool last, bool SP = false>
__device__ void attn_bwd_chunk(Smem& sm, const AttnPre& a, int c, float* scratch, int qsel = -1,
                               float* __restrict__ dqkv = nullptr, int b0 = 0, float* __restrict__ kvc = nullptr,
                               int kblk = 0) {
    const int o8 = tid_x() & 7, hh = (tid_x() >> 3) & 3, p = tid_x() >> 5;
    const int d0 = hh * HD + 2 * o8;
    const int col = 64 * c + d0;
    f32x2 k[S], v[S], dk[S], dv[S];
    bool msk[S];
    f32x2 sdq = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < S; ++j) {
        k[j] = a.k[j];
        v[j] = a.v[j];
        msk[j] = sm.mask[p * S + j] != 0;
        dk[j] = f32x2{0.f, 0.f};
        dv[j] = f32x2{0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < S; ++i) {
        f32x2 dq = {0.f, 0.f};
        if (qsel >= 0 ? i == qsel : (!last || i == S - 1)) {
            // the scores' 1/sqrt(16) on the query (q4 = q / 4: exact), so dk[j] += ds q = (ds 4) q4 and
            // dq = (sum_j (ds 4) k_j) / 4 -- the same values as scaling each score and each ds, without
            // the 2 S multiplies (EXP=104, A/B build: that form)
            constexpr bool kQ4 = UAVHIP_EXP != 104;
            const f32x2 q = a.q[i], q4 = kQ4 ? q * 0.25f : q;
            const f32x2 g = ld2(sm.ctx + (i * SPW + p) * LDH + col);
            float pr[S], dp[S];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                const float part = sum8(q4.x * k[j].x + q4.y * k[j].y);
                pr[j] = msk[j] ? -INFINITY : (kQ4 ? part : part * 0.25f);
                mx = (kQ4 && j == 0) ? pr[j] : fmaxf(mx, pr[j]);
            }
            float den = 0.f;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                pr[j] = __expf(pr[j] - mx);
                den = (kQ4 && j == 0) ? pr[j] : den + pr[j];
            }
            const float inv = att_recip(den);
            float sdp = 0.f;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                pr[j] *= inv;
                dp[j] = sum8(g.x * v[j].x + g.y * v[j].y);
                sdp += pr[j] * dp[j];
            }
#pragma unroll
            for (int j = 0; j < S; ++j) {
                const float ds = kQ4 ? pr[j] * (dp[j] - sdp) : pr[j] * (dp[j] - sdp) * 0.25f;
                dq += ds * k[j];
                dk[j] += ds * q4;
                dv[j] += pr[j] * g;
            }
            if (kQ4) dq *= 0.25f;
            sdq += dq;
        }
        if (!SP || (qsel >= 0 ? i == qsel : (!last || i == S - 1))) attn_out2(sm, dqkv, b0, i * SPW + p, d0, 0, c, dq, SP);
    }
    f32x2 sk = {0.f, 0.f}, sv = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < S; ++j) {
        attn_out2(sm, dqkv, b0, j * SPW + p, d0, 1, c, dk[j], SP, kvc, kblk);
        attn_out2(sm, dqkv, b0, j * SPW + p, d0, 2, c, dv[j], SP, kvc, kblk);
        sk += dk[j];
        sv += dv[j];
    }
    // the wave's two samples are lanes 32 apart
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        sdq[e] = add_xor32(sdq[e]);
        sk[e] = add_xor32(sk[e]);
        sv[e] = add_xor32(sv[e]);
    }
    if ((tid_x() & 63) < 32) {
        float* row = scratch + (tid_x() >> 6) * 3 * 64;
        st2(row + d0, sdq);
        st2(row + 64 + d0, sk);
        st2(row + 128 + d0, sv);
    }
}

// Backward of one post-LN encoder layer. On entry sm.h holds dL/d(layer output) for the tokens
// >= qtok0; on exit sm.h holds dL/d(layer input) for all 80 tokens. Ends with a barrier.
// The embedding backward's global inputs (embed_bwd): this thread's 20 embedding values (the ReLU
// mask) and one float4 of the input windows, loaded by the layer-0 backward right after its last
// GEMM (every weight load of the layer issued: nothing waits behind them), so their latency hides
// under the layer's final residual pass and barrier.
struct EmbBwdPre {
    float ev[TOK / 4];
    f32x4 xv;
};
__device__ __forceinline__ void embed_bwd_load(EmbBwdPre& ep, const float* __restrict__ e, const float* __restrict__ xg,
                                               int b0) {
    const int f = tid_x() & (D - 1), grp = tid_x() >> 7;
#pragma unroll
    for (int i = 0; i < TOK / 4; ++i) ep.ev[i] = e[(size_t)trow(grp + 4 * i, b0) * D + f];
    const int i = tid_x();
    ep.xv = i < TOK * LDX / 4 ? ld4(xg + (size_t)trow(i / (LDX / 4), b0) * 16 + 4 * (i % (LDX / 4)))
                              : f32x4{0.f, 0.f, 0.f, 0.f};
}

enum { kBwdFull = 0, kBwdNoDx = 1, kBwdPos = 2 };  // bwd_layer's MODE (see bwd_layer)
constexpr bool kBwdSplit = true;  // K6 (k_policy_backward) on split products
constexpr bool kPsSplit = true;   // the K7 position-split kernels (k_ps_f1..f3, k_ps_b1..b3) on split products
static_assert(kTrainF32LayerCopies || (kTrainSplit && kBwdSplit && kPsSplit),
              "a training kernel on f32 products reads the fp32 layer copies policy_pack_train leaves NaN");
// The layer backward as split products (bwd_layer<..., SP>): the same phases, barriers and outputs
// as the f32 path below, for every MODE.
template <int trunk, int layer, bool last, int TB, class F, int MODE>
__device__ void bwd_layer_split(Smem& sm, const float* __restrict__ P, const float* __restrict__ PT, const BwdLayerIO& io,
                                int b0, EmbBwdPre* ep, const float* e_emb, const float* xg, const LnBwdPre* ln2_pre,
                                F next_load, int liT, int qt, int prow, float* __restrict__ kvc) {
    constexpr int CTQ = (last || MODE == kBwdPos) ? 1 : S;
    const int qtok0 = last ? (S - 1) * SPW : (MODE == kBwdPos ? qt : 0), qtok1 = qtok0 + SPW * CTQ;
    const int qsel = MODE == kBwdPos ? qt / SPW : -1;
    (void)liT;  // PT is this layer's packedT (the caller's offset): its split copy at PT + kTSplit
    const int sWin = kTSplit + kTWin, sWo = kTSplit + kTWo, sW1 = kTSplit + kTW1, sW2 = kTSplit + kTW2;
    const int wv = tid_x() >> 6, l = lane_id(), i16 = l & 15, g = l >> 4;
    const int fo = 16 * wv + 4 * g;
    const int blk = prow >= 0 ? prow : b0 / SPW;  // this workgroup's partial rows
    float* bias = io.bpart + (size_t)blk * kBiasPart;
    _Float16* const hp = reinterpret_cast<_Float16*>(sm.h);
    _Float16* const bp = reinterpret_cast<_Float16*>(sm.big);
    _Float16* const cp = reinterpret_cast<_Float16*>(sm.ctx);
    auto unsplit = [](const _Float16* x, int o) {  // x1 + 2^-11 x2 of 4 halves at o
        const f16x4 a = *reinterpret_cast<const f16x4*>(x + o), b = *reinterpret_cast<const f16x4*>(x + o + kPlane);
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (float)a[j] + (float)b[j] * kLoScale;
        return v;
    };
    // LN2 backward: sm.h -> df planes in sm.ctx
    HPre<2> pa = hprefetch<2>(PT, sW2, D, 16 * wv, 0);
    LnBwdPre lnp;
    if (ln2_pre) lnp = *ln2_pre;
    else ln_bwd_load(lnp, io.xhat2, io.rstd2, P + kOffs.o[layer_param(trunk, layer, N2W)], qtok0, b0, last, qtok1);
    ln_bwd_lds<true>(sm.h, sm.ctx, lnp, io.df, io.ln2_part + (size_t)blk * 2 * D, bias + kBiasL2, qtok0, b0, last,
                     sm.big, qtok1);
    BTR(TB + 1);
    __syncthreads();
    BTR(TB + 2);
    // du = relu'(u) (W2^T df): wave wv owns hidden tiles 16 wv (-> big planes) and 128 + 16 wv (-> h planes)
    HPre<2> pb;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int row = 128 * t + 16 * wv;
        f32x4 hi[CTQ], lo[CTQ], uu[CTQ];
#pragma unroll
        for (int ct = 0; ct < CTQ; ++ct)
            uu[ct] = ld4(io.u + (size_t)orow(qtok0 + 16 * ct + i16, b0, last) * FF + row + 4 * g);
        zero(hi);
        zero(lo);
        if (t == 0) {
            hgemm_tile<CTQ, 2>(hi, lo, pa, PT, sW2, D, row, 0, cp, qtok0);
            pb = hprefetch<2>(PT, sW2, D, 128 + 16 * wv, 0);
        } else {
            hgemm_tile<CTQ, 2>(hi, lo, pb, PT, sW2, D, row, 0, cp, qtok0);
            pa = hprefetch<2>(PT, sW1, FF, 16 * wv, 0);
        }
        _Float16* dstp = t ? hp : bp;
        f32x4 sd = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ct = 0; ct < CTQ; ++ct) {
            const int tok = qtok0 + 16 * ct + i16;
            const size_t r = (size_t)orow(tok, b0, last);
            const f32x4 u = uu[ct];
            f32x4 d = hi[ct] + lo[ct] * kLoScale;
            d.x = u.x > 0.f ? d.x : 0.f; d.y = u.y > 0.f ? d.y : 0.f;
            d.z = u.z > 0.f ? d.z : 0.f; d.w = u.w > 0.f ? d.w : 0.f;
            dy_st4(io.du + r * FF + row + 4 * g, d);
            hsplit_store(dstp, psw(tok, fo), d);
            sd += d;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) sd[e] = row16_sum(sd[e]);
        if (i16 == 0) st4(bias + kBiasL1 + row + 4 * g, sd);
    }
    BTR(TB + 3);
    __syncthreads();
    BTR(TB + 4);
    // dh1 = df + W1^T du (K = 256: hidden 0-127 in big, 128-255 in h) -> sm.ctx in fp32, after every
    // lane has read its df (the fp32 rows overlap the planes)
    {
        f32x4 hi[CTQ], lo[CTQ];
        zero(hi);
        zero(lo);
        hgemm_tile<CTQ, 2>(hi, lo, pa, PT, sW1, FF, 16 * wv, 0, bp, qtok0);
        hgemm_tile<CTQ, 2>(hi, lo, hprefetch<2>(PT, sW1, FF, 16 * wv, 128), PT, sW1, FF, 16 * wv, 128, hp, qtok0);
#pragma unroll
        for (int ct = 0; ct < CTQ; ++ct) hi[ct] = hi[ct] + lo[ct] * kLoScale + unsplit(cp, psw((qtok0 + 16 * ct + i16), fo));
        __syncthreads();
#pragma unroll
        for (int ct = 0; ct < CTQ; ++ct) st4(sm.ctx + (qtok0 + 16 * ct + i16) * LDH + fo, hi[ct]);
    }
    pa = hprefetch<2>(PT, sWo, D, 16 * wv, 0);
    ln_bwd_load(lnp, io.xhat1, io.rstd1, P + kOffs.o[layer_param(trunk, layer, N1W)], qtok0, b0, last, qtok1);
    AttnPre ap;
    attn_bwd_load<last>(ap, io.qkv, 0, b0, qsel);
    // the position-split modes have no W_in^T GEMM to hide chunk 1's Q / K / V rows behind: both
    // chunks' rows are loaded here (K6 loads chunk 1's behind chunk 0's weight loads, below)
    BTR(TB + 5);
    __syncthreads();
    BTR(TB + 6);
    // LN1 backward: sm.ctx -> dz1 planes in sm.h
    ln_bwd_lds<true>(sm.ctx, sm.h, lnp, io.dz1, io.ln1_part + (size_t)blk * 2 * D, bias + kBiasOut, qtok0, b0, last,
                     sm.big, qtok1);
    BTR(TB + 7);
    __syncthreads();
    BTR(TB + 8);
    // d(attention output) = Wo^T dz1 -> sm.ctx (fp32: the attention backward's operand)
    {
        f32x4 hi[CTQ], lo[CTQ];
        zero(hi);
        zero(lo);
        hgemm_tile<CTQ, 2>(hi, lo, pa, PT, sWo, D, 16 * wv, 0, hp, qtok0);
#pragma unroll
        for (int ct = 0; ct < CTQ; ++ct) st4(sm.ctx + (qtok0 + 16 * ct + i16) * LDH + fo, hi[ct] + lo[ct] * kLoScale);
    }
    BTR(TB + 9);
    __syncthreads();
    BTR(TB + 10);
    // attention backward per chunk of 4 heads, dh_in += W_in^T [dq | dk | dv] of the chunk (K = 3 x 64)
    f32x4 hi[S], lo[S];
    zero(hi);
    zero(lo);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        [[maybe_unused]] HPre<2> pw;
        if constexpr (MODE == kBwdFull) pw = hprefetch<2>(PT, sWin, 3 * D, 16 * wv, 64 * c);
        attn_bwd_chunk<last, true>(sm, ap, c, sm.scr, qsel, io.dqkv, b0, MODE == kBwdPos ? kvc : nullptr, blk);
        __syncthreads();
        BTR(TB + 11 + 2 * c);
        if (tid_x() < 3 * 64) {  // in_proj bias partial of the chunk: the 8 wave rows of sm.scr
            const int i = tid_x();
            float v = 0.f;
#pragma unroll
            for (int w = 0; w < NW; ++w) v += sm.scr[w * 192 + i];
            bias[kBiasIn + (i >> 6) * D + 64 * c + (i & 63)] = v;
        }
        if constexpr (MODE != kBwdFull) {  // the per-position kernels form dL/d(layer input)
            if (c == 0) attn_bwd_load<last>(ap, io.qkv, 1, b0, qsel);
            if (c == 0) __syncthreads();  // sm.scr is rewritten by chunk 1
            continue;
        }
        const HPre<2> pw1 = hprefetch<2>(PT, sWin, 3 * D, 16 * wv, D + 64 * c);
        const HPre<2> pw2 = hprefetch<2>(PT, sWin, 3 * D, 16 * wv, 2 * D + 64 * c);
        if (last) {  // dq is zero outside the query tile: W_in,q^T dq only for column tile 4
            f32x4 h1[1] = {hi[S - 1]}, l1[1] = {lo[S - 1]};
            hgemm_tile<1, 2, 2, kLdbP, kPlaneB>(h1, l1, pw, PT, sWin, 3 * D, 16 * wv, 64 * c, bp, (S - 1) * SPW);
            hi[S - 1] = h1[0];
            lo[S - 1] = l1[0];
        } else {
            hgemm_tile<S, 2, 2, kLdbP, kPlaneB>(hi, lo, pw, PT, sWin, 3 * D, 16 * wv, 64 * c, bp, 0);
        }
        hgemm_tile<S, 2, 2, kLdbP, kPlaneB>(hi, lo, pw1, PT, sWin, 3 * D, 16 * wv, D + 64 * c, bp + 64, 0);
        hgemm_tile<S, 2, 2, kLdbP, kPlaneB>(hi, lo, pw2, PT, sWin, 3 * D, 16 * wv, 2 * D + 64 * c, bp + 128, 0);
        if (c == 0) attn_bwd_load<last>(ap, io.qkv, 1, b0, qsel);  // behind every weight load of the chunk
        if (c == 0) __syncthreads();  // big is rewritten by chunk 1
        BTR(TB + 12 + 2 * c);
    }
    if constexpr (MODE != kBwdFull) return;
    if (layer == 0 && ep) embed_bwd_load(*ep, e_emb, xg, b0);
    next_load();
    // + dz1 on the rows that carried the residual -> sm.h (fp32, after every lane has read its dz1)
    f32x4 res[S];
#pragma unroll
    for (int ct = 0; ct < S; ++ct) {
        const int tok = 16 * ct + i16;
        res[ct] = tok >= qtok0 ? unsplit(hp, psw(tok, fo)) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
#pragma unroll
    for (int ct = 0; ct < S; ++ct) st4(sm.h + (16 * ct + i16) * LDH + fo, hi[ct] + lo[ct] * kLoScale + res[ct]);
    __syncthreads();
    BTR(TB + 15);
}

// ln2_pre: this layer's LN2-backward operands, already loaded by the caller (nullptr: load here);
// next_load: issues the next phase's global loads behind this layer's last weight loads.
// MODE (the position-split training step, K7 below): kBwdFull = the whole layer; kBwdNoDx = stop after
// the attention backward (dqkv rows and bias partials written; no W_in^T GEMM, no residual -- the
// per-position kernels form dL/d(layer input)); kBwdPos = a full layer for the 16 query tokens of
// ONE window position (tokens [qt, qt + 16), [b * 5 + s] rows, partial row prow): its dq rows go to
// dqkv, its contributions to every position's dk / dv to kvc ([prow][80 tokens][dk 128 | dv 128]).
// SP (kBwdFull only): every dX GEMM as split products on the f16 MFMA -- A = the transposed split
// copies (PT + kTSplit), B = planes the producing epilogue writes: df (LN2 backward -> sm.ctx), du
// (-> sm.big / sm.h), dz1 (LN1 backward -> sm.h), dq | dk | dv (attention backward -> sm.big, rows of
// kLdbP halves, attn_out2); the residual terms read back from planes are x1 + 2^-11 x2.
template <int trunk, int layer, bool last, int TB, class F = NoHook, int MODE = kBwdFull, bool SP = false>
__device__ void bwd_layer(Smem& sm, const float* __restrict__ P, const float* __restrict__ PT, const BwdLayerIO& io,
                          int b0, EmbBwdPre* ep = nullptr, const float* e_emb = nullptr, const float* xg = nullptr,
                          const LnBwdPre* ln2_pre = nullptr, F next_load = F{}, int qt = 0, int prow = -1,
                          float* __restrict__ kvc = nullptr) {
    constexpr int liT = (trunk == kActorTrunk ? 0 : 1 + layer) * kLayerT;  // this layer's packedT offset
    BTR(TB);
    static_assert(MODE != kBwdPos || !last, "position split: full layers only");
    constexpr int CTQ = (last || MODE == kBwdPos) ? 1 : S;
    constexpr int DQ = depth<CTQ>();
    const int qtok0 = last ? (S - 1) * SPW : (MODE == kBwdPos ? qt : 0);
    const int qtok1 = qtok0 + SPW * CTQ;
    const int qsel = MODE == kBwdPos ? qt / SPW : -1;
    const float* WinT = PT + kTWin;
    const float* WoT = PT + kTWo;
    const float* W1T = PT + kTW1;
    const float* W2T = PT + kTW2;
    const int wv = tid_x() >> 6, l = lane_id(), i16 = l & 15, g = l >> 4;
    const int fo = 16 * wv + 4 * g;  // this lane's 4 output features of a 16-row tile of wave wv
    const int blk = prow >= 0 ? prow : b0 / SPW;  // this workgroup's partial rows
    float* bias = io.bpart + (size_t)blk * kBiasPart;  // this workgroup's bias partials

    if constexpr (SP) {
        bwd_layer_split<trunk, layer, last, TB, F, MODE>(sm, P, PT, io, b0, ep, e_emb, xg, ln2_pre, next_load, liT, qt,
                                                         prow, kvc);
        return;
    } else {
    // LN2 backward: sm.h -> sm.ctx (= df)
    APre<DQ> pa = prefetch<DQ>(W2T, D, 16 * wv, 0);
    LnBwdPre lnp;
    if (ln2_pre) lnp = *ln2_pre;
    else ln_bwd_load(lnp, io.xhat2, io.rstd2, P + kOffs.o[layer_param(trunk, layer, N2W)], qtok0, b0, last, qtok1);
    ln_bwd_lds(sm.h, sm.ctx, lnp, io.df, io.ln2_part + (size_t)blk * 2 * D, bias + kBiasL2, qtok0, b0, last,
               sm.big, qtok1);
    BTR(TB + 1);
    __syncthreads();
    BTR(TB + 2);
    // du = relu'(u) (W2^T df): 256 hidden features, wave wv owns tiles 16 wv (-> big) and 128 + 16 wv (-> h)
    // the next GEMM's first weight blocks are loaded before each tile's du stores (a load issued
    // behind a store burst waits for the whole burst)
    APre<DQ> pb;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int row = 128 * t + 16 * wv;
        f32x4 acc[CTQ], uu[CTQ];  // u (for the ReLU mask) loaded ahead of the GEMM
#pragma unroll
        for (int ct = 0; ct < CTQ; ++ct)
            uu[ct] = ld4(io.u + (size_t)orow(qtok0 + 16 * ct + i16, b0, last) * FF + row + 4 * g);
        zero(acc);
        if (t == 0) {
            gemm_tile<CTQ, DQ>(acc, pa, W2T, D, row, 0, sm.ctx, LDH, qtok0);
            pb = prefetch<DQ>(W2T, D, 128 + 16 * wv, 0);
        } else {
            gemm_tile<CTQ, DQ>(acc, pb, W2T, D, row, 0, sm.ctx, LDH, qtok0);
            pa = prefetch<DQ>(W1T, FF, 16 * wv, 0);
        }
        float* lds = t ? sm.h : sm.big;
        f32x4 sd = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ct = 0; ct < CTQ; ++ct) {
            const int tok = qtok0 + 16 * ct + i16;
            const size_t r = (size_t)orow(tok, b0, last);
            const f32x4 u = uu[ct];
            f32x4 d = acc[ct];
            d.x = u.x > 0.f ? d.x : 0.f; d.y = u.y > 0.f ? d.y : 0.f;
            d.z = u.z > 0.f ? d.z : 0.f; d.w = u.w > 0.f ? d.w : 0.f;
            dy_st4(io.du + r * FF + row + 4 * g, d);
            st4(lds + tok * LDH + fo, d);
            sd += d;
        }
        // linear1 bias partial: sum over the tokens (the 16 lanes of a row, then the column tiles)
#pragma unroll
        for (int e = 0; e < 4; ++e) sd[e] = row16_sum(sd[e]);
        if (i16 == 0) st4(bias + kBiasL1 + row + 4 * g, sd);
    }
    BTR(TB + 3);
    __syncthreads();
    BTR(TB + 4);
    // dh1 = df + W1^T du (K = 256: hidden 0-127 in big, 128-255 in h) -> sm.ctx in place
    {
        f32x4 acc[CTQ];
        zero(acc);
        gemm_tile<CTQ, DQ>(acc, pa, W1T, FF, 16 * wv, 0, sm.big, LDF, qtok0);
        gemm_tile<CTQ, DQ>(acc, prefetch<DQ>(W1T, FF, 16 * wv, 128), W1T, FF, 16 * wv, 128, sm.h, LDH, qtok0);
#pragma unroll
        for (int ct = 0; ct < CTQ; ++ct) {
            float* q = sm.ctx + (qtok0 + 16 * ct + i16) * LDH + fo;
            st4(q, acc[ct] + ld4(q));
        }
    }
    pa = prefetch<DQ>(WoT, D, 16 * wv, 0);
    // LN1 backward's operands, then chunk 0's Q / K / V for the attention backward: their HBM
    // latency hides under the residual pass / barrier and LN1 backward
    ln_bwd_load(lnp, io.xhat1, io.rstd1, P + kOffs.o[layer_param(trunk, layer, N1W)], qtok0, b0, last, qtok1);
    AttnPre ap;
    attn_bwd_load<last>(ap, io.qkv, 0, b0, qsel);
    BTR(TB + 5);
    __syncthreads();
    BTR(TB + 6);
    // LN1 backward: sm.ctx -> sm.h (= dz1)
    ln_bwd_lds(sm.ctx, sm.h, lnp, io.dz1, io.ln1_part + (size_t)blk * 2 * D, bias + kBiasOut, qtok0, b0, last,
               sm.big, qtok1);
    BTR(TB + 7);
    __syncthreads();
    BTR(TB + 8);
    // d(attention output) = Wo^T dz1 -> sm.ctx
    {
        f32x4 acc[CTQ];
        zero(acc);
        gemm_tile<CTQ, DQ>(acc, pa, WoT, D, 16 * wv, 0, sm.h, LDH, qtok0);
#pragma unroll
        for (int ct = 0; ct < CTQ; ++ct) st4(sm.ctx + (qtok0 + 16 * ct + i16) * LDH + fo, acc[ct]);
    }
    BTR(TB + 9);
    __syncthreads();
    BTR(TB + 10);
    // attention backward per chunk of 4 heads, dh_in += Win^T [dq | dk | dv] of the chunk (K = 3 x 64)
    constexpr bool kDx = MODE == kBwdFull;
    f32x4 acc[S];
    zero(acc);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        [[maybe_unused]] APre<2> pw;
        if constexpr (kDx) pw = prefetch<2>(WinT, 3 * D, 16 * wv, 64 * c);
        attn_bwd_chunk<last>(sm, ap, c, sm.scr, qsel);
        __syncthreads();
        BTR(TB + 11 + 2 * c);
        if (tid_x() < 3 * 64) {  // in_proj bias partial of the chunk: the 8 wave rows of sm.scr
            const int i = tid_x();
            float v = 0.f;
#pragma unroll
            for (int w = 0; w < NW; ++w) v += sm.scr[w * 192 + i];
            bias[kBiasIn + (i >> 6) * D + 64 * c + (i & 63)] = v;
        }
        // first weight blocks of the chunk's K and V parts, loaded ahead of the stores below (the
        // vector memory counter retires in order: loads behind a store burst wait for it)
        [[maybe_unused]] APre<2> pw1, pw2;
        if constexpr (kDx) {
            pw1 = prefetch<2>(WinT, 3 * D, 16 * wv, D + 64 * c);
            pw2 = prefetch<2>(WinT, 3 * D, 16 * wv, 2 * D + 64 * c);
        }
        // dq | dk | dv of the chunk -> dqkv rows: 256-byte row segments, float4 per thread
        for (int i = tid_x(); i < TOK * 48; i += NTHR) {
            const int tok = i / 48, r = i - tok * 48, part = r >> 4, q = r & 15;
            if (part == 0 && (tok < qtok0 || tok >= qtok1)) continue;  // dq only on the query rows
            const f32x4 v = ld4(sm.big + tok * LDB + part * 64 + 4 * q);
            if (MODE == kBwdPos && part > 0)  // this query position's share of every position's dk / dv
                st4(kvc + ((size_t)blk * TOK + tok) * 2 * D + (part - 1) * D + 64 * c + 4 * q, v);
            else
                dy_st4(io.dqkv + (size_t)trow(tok, b0) * 3 * D + part * D + 64 * c + 4 * q, v);
        }
        if constexpr (kDx) {
            if (last) {  // dq is zero outside the query tile: Win_q^T dq only for column tile 4
                f32x4 a1[1] = {acc[S - 1]};
                gemm_tile<1, 2, 4>(a1, pw, WinT, 3 * D, 16 * wv, 64 * c, sm.big, LDB, (S - 1) * SPW);
                acc[S - 1] = a1[0];
            } else {
                gemm_tile<S, 2, 4>(acc, pw, WinT, 3 * D, 16 * wv, 64 * c, sm.big, LDB, 0);
            }
            gemm_tile<S, 2, 4>(acc, pw1, WinT, 3 * D, 16 * wv, D + 64 * c, sm.big + 64, LDB, 0);
            gemm_tile<S, 2, 4>(acc, pw2, WinT, 3 * D, 16 * wv, 2 * D + 64 * c, sm.big + 128, LDB, 0);
        }
        if (c == 0) attn_bwd_load<last>(ap, io.qkv, 1, b0, qsel);  // behind every weight load of the chunk
        if (c == 0) __syncthreads();  // big is rewritten by chunk 1
        BTR(TB + 12 + 2 * c);
    }
    if constexpr (!kDx) return;
    if (layer == 0 && ep) embed_bwd_load(*ep, e_emb, xg, b0);
    next_load();
    // + dz1 on the rows that carried the residual -> sm.h
#pragma unroll
    for (int ct = 0; ct < S; ++ct) {
        const int tok = 16 * ct + i16;
        float* q = sm.h + tok * LDH + fo;
        st4(q, tok >= qtok0 ? acc[ct] + ld4(q) : acc[ct]);
    }
    __syncthreads();
    BTR(TB + 15);
    }
}

// Embedding backward from sm.h = dL/d(h0) (80 tokens): h0 = relu(We x + be) + pos. Thread =
// (feature, token group of 20); partials reduced over the 4 groups through sm.big -> part [2560]
// in the parameters' order (pos | We | be).
__device__ void embed_bwd(Smem& sm, const EmbBwdPre& ep, float* __restrict__ part, int tb = 55) {
    const int f = tid_x() & (D - 1), grp = tid_x() >> 7;
    if (tid_x() < TOK * LDX / 4) st4(sm.x + 4 * tid_x(), ep.xv);  // input windows (sm.x was scratch)
    __syncthreads();
    BTR(tb);
    float acc[IN + 1 + S];
#pragma unroll
    for (int v = 0; v < IN + 1 + S; ++v) acc[v] = 0.f;
#pragma unroll
    for (int i = 0; i < TOK / 4; ++i) {
        const int tok = grp + 4 * i;  // position tok / 16 = i / 4
        const float gv = sm.h[tok * LDH + f];
        acc[IN + 1 + i / 4] += gv;
        const float gp = ep.ev[i] > 0.f ? gv : 0.f;
        acc[IN] += gp;
        float xr[LDX];  // the token's window row: 4 broadcast b128 reads
#pragma unroll
        for (int q = 0; q < LDX / 4; ++q) {
            const f32x4 x4 = ld4(sm.x + tok * LDX + 4 * q);
            xr[4 * q] = x4.x; xr[4 * q + 1] = x4.y; xr[4 * q + 2] = x4.z; xr[4 * q + 3] = x4.w;
        }
#pragma unroll
        for (int k = 0; k < IN; ++k) acc[k] += gp * xr[k];
    }
    constexpr int NV = IN + 1 + S;  // 20
#pragma unroll
    for (int v = 0; v < NV; ++v) sm.big[(grp * NV + v) * D + f] = acc[v];
    __syncthreads();
    BTR(tb + 1);
    for (int o = tid_x(); o < NV * D; o += NTHR) {
        const int v = o >> 7, ff = o & (D - 1);
        const float s = (sm.big[v * D + ff] + sm.big[(NV + v) * D + ff]) +
                        (sm.big[(2 * NV + v) * D + ff] + sm.big[(3 * NV + v) * D + ff]);
        // state_dict order of the trunk's first parameters: pos [5][128] | We [128][14] | be [128]
        const int dst = v < IN ? S * D + ff * IN + v : (v == IN ? S * D + D * IN + ff : (v - IN - 1) * D + ff);
        part[dst] = s;
    }
}

// Loss gradients of ppo.py:148-169 per sample (torch's min / max / clamp backward conventions:
// ties send half the gradient to each side, clamp passes it on the closed interval), then the
// heads' backward: dz = relu'(z) (W2^T g) for both heads -> io.dz, LDS (actor: sm.z, critic:
// sm.ctx + 64, both [16][LDZ]), and the head.2 weight / bias partials of the 16 samples.
// role (trunk split): 0 both heads, 1 the actor head only, 2 the critic head only.
__device__ void heads_bwd(Smem& sm, const float* __restrict__ P, const BwdIO& io, int b0, int role) {
    const int blk = b0 / SPW;
    float* gs = sm.ctx;                  // [16][4]: dlogit0, dlogit1, dvalue
    float* dzc = sm.ctx + 64;            // critic dz rows
    float* zs = sm.big;                  // relu(head.0) rows of both heads [2][16][64]
    const float inv = 1.0f / (float)io.Bg;
    // the gradient path's 1/Bg pre-scaled by the power of two io.gscale (BwdIO::gscale): gradients
    // leave this function gscale x the loss's, bit for bit (power-of-two scaling commutes with every
    // rounding), and stay that way through the linear backward until k_reduce_grads' 1/gscale
    const float ginv = inv * io.gscale;
    // the critic's gradients additionally x 2^-k (k > 0 only when a value error of the minibatch
    // reaches 16): its per-sample gradient is ~ |v - R|, which returns of configs[4]'s scale and
    // beyond would carry past fp16's range in the split-product dX GEMMs. Every workgroup forms the
    // same k from the forward's per-block maxima (vpart); the critic's reductions undo it
    // (k_reduce_grads reads 2^k from gsc_out).
    // Every wave reduces the maxima itself (a few L2-resident loads per lane), so ck / ginv_c are the
    // same in every lane of the workgroup (wave 0 alone had them). ck saturates at 124
    // for an infinite maximum (2^-124 is still a normal float; a NaN maximum keeps ck = 0: the loss is
    // NaN then anyway).
    float vmx = 0.f;
    for (int i = tid_x() & 63; i < io.nvpart; i += 64) vmx = fmaxf(vmx, io.vpart[i]);
    vmx = wave_max(vmx);
    int vexp = 0;
    (void)frexpf(vmx, &vexp);
    const int ck = !(vmx >= 16.f) ? 0 : vmx < 3.0e38f ? vexp - 4 : 124;  // vmx 2^-ck in [8, 16)
    const float ginv_c = ginv * ldexpf(1.0f, -ck);
    if (tid_x() == 0 && blk == 0 && role != 1 && io.gsc_out) io.gsc_out[0] = ldexpf(1.0f, ck);
    // the four loss sums (used by wave 0 only): from the all-reduced buffer, or summed here from
    // the forward's workgroup partials with k_loss_sums' exact order (train.hip)
    // every global input issued before the first use: z rows (one float4 per thread), the head.2
    // weights of this thread's hidden unit j = tid % 64 (the dz loop below), the per-sample rows,
    // then the loss-sum partials four rows per thread at a time (a dependent chain of L2 round trips
    // before: the heads prologue took 10.7 k cycles of K6)
    const int zt = tid_x() >> 8, zp = (tid_x() >> 4) & 15, zq = tid_x() & 15;
    const f32x4 zr = ld4(io.z[zt] + (size_t)(b0 + zp) * HID + 4 * zq);
    const int jj = tid_x() % HID;
    const float* W2a = P + kOffs.o[kActorHead + 2];
    const float w2a0 = W2a[jj], w2a1 = W2a[HID + jj], w2c = P[kOffs.o[kCriticHead + 2] + jj];
    f32x4 oa = {0.f, 0.f, 0.f, 0.f}, ob = oa;
    if (tid_x() < SPW) {
        oa = ld4(io.smp + (size_t)(b0 + tid_x()) * 8);
        ob = ld4(io.smp + (size_t)(b0 + tid_x()) * 8 + 4);
    }
    float tot0, tot1, tot2, tot3;
    if (io.fpart) {
        f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
        if (tid_x() < 64) {  // row i's four sums, rows in k_loss_sums' order per lane
#pragma unroll 4
            for (int i = tid_x(); i < io.nfpart; i += 64) s4 += ld4(io.fpart + (size_t)i * 4);
#pragma unroll
            for (int c = 0; c < 4; ++c)
                s4[c] = add_xor32(add_xor16(add_ror8(add_ror4(add_xor2(add_xor1(s4[c]))))));
            if (blk == 0 && role != 2 && tid_x() == 0 && io.tot_out)
                for (int c = 0; c < 4; ++c) io.tot_out[c] = s4[c];
        }
        tot0 = s4[0]; tot1 = s4[1]; tot2 = s4[2]; tot3 = s4[3];
    } else {
        tot0 = io.tot[0]; tot1 = io.tot[1]; tot2 = io.tot[2]; tot3 = io.tot[3];
    }
    BTR(59);
    st4(zs + (zt * SPW + zp) * HID + 4 * zq, zr);
    if (tid_x() < SPW) {
        const int p = tid_x();
        const float o[8] = {oa.x, oa.y, oa.z, oa.w, ob.x, ob.y, ob.z, ob.w};
        const int act = o[0] > 0.f;
        const bool pad = o[0] < 0.f;  // padding row (idx < 0): zero output gradients
        const CatVals c = categorical(o[5], o[6]);
        const float logp = act ? c.lc1 : c.lc0;
        const float ratio = expf(logp - o[1]);
        const float A = o[4], lo = 1.f - io.eps_clip, hi = 1.f + io.eps_clip;
        const float s1 = ratio * A;
        const float s2 = fminf(fmaxf(ratio, lo), hi) * A;
        const float gmin = -ginv;  // d(-mean(min)) / d min_i (x gscale)
        const float g1 = s1 < s2 ? gmin : (s1 == s2 ? 0.5f * gmin : 0.f);
        const float g2 = s2 < s1 ? gmin : (s1 == s2 ? 0.5f * gmin : 0.f);
        const float gr = g1 * A + ((ratio >= lo && ratio <= hi) ? g2 * A : 0.f);
        const float glogp = gr * ratio;
        const float gent = -io.entropy_coef * ginv;
        // back through lc = log(clamp(p)), ent = -sum(lc * p), p = y / s, s = y0 + y1, y = softmax
        float glc0 = -gent * c.p0, glc1 = -gent * c.p1;
        if (act) glc1 += glogp; else glc0 += glogp;
        const float eps = 1.1920928955078125e-07f;
        const float gp0 = -gent * c.lc0 + ((c.p0 >= eps && c.p0 <= 1.f - eps) ? glc0 / c.c0 : 0.f);
        const float gp1 = -gent * c.lc1 + ((c.p1 >= eps && c.p1 <= 1.f - eps) ? glc1 / c.c1 : 0.f);
        const float gsum = -(gp0 * c.y0 + gp1 * c.y1) / (c.s * c.s);
        const float gy0 = gp0 / c.s + gsum, gy1 = gp1 / c.s + gsum;
        const float dot = gy0 * c.y0 + gy1 * c.y1;
        // value: 0.5 * max(mean((v-R)^2), mean((vc-R)^2))
        const float L1 = tot1 * inv, L2 = tot2 * inv;
        const float v = o[7], R = o[3], ov = o[2];
        const float dv = v - ov;
        const float vc = ov + fminf(fmaxf(dv, -io.eps_clip), io.eps_clip);
        const float w1 = L1 > L2 ? 1.f : (L1 == L2 ? 0.5f : 0.f);
        const float w2 = L2 > L1 ? 1.f : (L1 == L2 ? 0.5f : 0.f);
        gs[4 * p + 0] = pad ? 0.f : c.y0 * (gy0 - dot);
        gs[4 * p + 1] = pad ? 0.f : c.y1 * (gy1 - dot);
        gs[4 * p + 2] = pad ? 0.f : io.value_coef * (w1 * 2.f * (v - R) * ginv_c +
                                         ((dv >= -io.eps_clip && dv <= io.eps_clip) ? w2 * 2.f * (vc - R) * ginv_c : 0.f));
        if (p == 0 && blk == 0 && role != 2 && io.stats) {
            io.stats[0] += (double)(-tot0 * inv);
            io.stats[1] += (double)fmaxf(L1, L2);
            io.stats[2] += (double)(tot3 * inv);
            io.stats[3] += 1.0;
        }
    }
    __syncthreads();
    BTR(60);
    static_assert(NTHR % HID == 0, "dz loop: j = tid % 64 for every i");
    for (int i = tid_x(); i < 2 * SPW * HID; i += NTHR) {
        const int trunk = i / (SPW * HID), p = (i / HID) % SPW, j = i % HID;
        if (role == 1 + (trunk ^ 1)) continue;  // the other role's head
        const float z = zs[(trunk * SPW + p) * HID + j];
        const float g = trunk ? w2c * gs[4 * p + 2] : w2a0 * gs[4 * p] + w2a1 * gs[4 * p + 1];
        const float dz = z > 0.f ? g : 0.f;
        io.dz[trunk][(size_t)(b0 + p) * HID + j] = dz;
        (trunk ? dzc : sm.z)[p * LDZ + j] = dz;
    }
    __syncthreads();
    BTR(61);
    // head.0 bias partials (sum over the 16 samples of dz, from LDS)
    if (tid_x() < 2 * HID && role != 1 + (tid_x() / HID ^ 1)) {
        const int trunk = tid_x() / HID, j = tid_x() % HID;
        const float* d = trunk ? dzc : sm.z;
        float acc = 0.f;
        for (int p = 0; p < SPW; ++p) acc += d[p * LDZ + j];
        io.hpart[(size_t)blk * kHeadPart + kHeadB0 + tid_x()] = acc;
    }
    // head.2 partials, summed over the 16 samples in order: dW2[o][j] = sum g_o z_j, db2[o] = sum g_o
    // [0, 2 HID + 2): actor head.2, [2 HID + 2, 3 HID + 3): critic head.2, then padding (actor role)
    if (tid_x() < kHeadB0 && role != ((tid_x() >= 2 * HID + 2 && tid_x() < 3 * HID + 3) ? 1 : 2)) {
        const int i = tid_x();
        float acc = 0.f;
        if (i < 2 * HID) {
            const int o = i / HID, j = i % HID;
            for (int p = 0; p < SPW; ++p) acc += gs[4 * p + o] * zs[p * HID + j];
        } else if (i < 2 * HID + 2) {
            for (int p = 0; p < SPW; ++p) acc += gs[4 * p + i - 2 * HID];
        } else if (i < 3 * HID + 2) {
            const int j = i - 2 * HID - 2;
            for (int p = 0; p < SPW; ++p) acc += gs[4 * p + 2] * zs[(SPW + p) * HID + j];
        } else if (i < 3 * HID + 3) {
            for (int p = 0; p < SPW; ++p) acc += gs[4 * p + 2];
        }
        io.hpart[(size_t)blk * kHeadPart + i] = acc;
    }
}

// dL/d(trunk output) of the 16 samples = head.0^T dz (MFMA, K = 64; one 16-feature tile per
// wave) -> sm.h rows of column tile 4, the top gradient of the trunk's last layer.
__device__ __forceinline__ void head_input_grad(Smem& sm, const float* __restrict__ W0T, const float* dz) {
    const int wv = tid_x() >> 6, l = lane_id(), i16 = l & 15, g = l >> 4;
    f32x4 acc[1];
    zero(acc);
    gemm_tile<1, 4, 4>(acc, prefetch<4>(W0T, HID, 16 * wv, 0), W0T, HID, 16 * wv, 0, dz, LDZ, 0);
    st4(sm.h + ((S - 1) * SPW + i16) * LDH + 16 * wv + 4 * g, acc[0]);
}

__global__ __launch_bounds__(NTHR) void k_policy_backward(const float* __restrict__ P, const float* __restrict__ PT,
                                                          const BwdIO io) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    // the younger half (waves 4-7, the arbitration loser of every phase) at priority 1
    if (tid_x() >= NTHR / 2) __builtin_amdgcn_s_setprio(1);
    // trunk split (BwdIO::split): workgroups [0, split) the actor head + trunk, then the critic's
    int blk = blockIdx.x, role = 0;
    if (io.split) {
        role = blk < io.split ? 1 : 2;
        if (role == 2) blk -= io.split;
    }
    const int b0 = blk * SPW;
    if (tid_x() < SPW * S) sm.mask[tid_x()] = io.mask[(size_t)b0 * S + tid_x()] != 0.f;
    BTR(0);
    heads_bwd(sm, P, io, b0, role);
    __syncthreads();
    BTR(1);
    // Trunk order (BwdIO::mix): the actor and critic trunks are independent below the heads, so
    // every other group of 8 workgroups (one per XCD) runs the actor first: at any time half the
    // chip is in the other trunk's phases, and the HBM-heavy phases of one overlap the compute of
    // the other instead of all 256 workgroups streaming at once. The critic's dz rows (sm.ctx + 64,
    // clobbered by the actor's layer) come back from io.dz[1], which heads_bwd wrote with them.
    const bool actor_first = role == 0 && io.mix && ((blk >> 3) & 1);
    // actor: head.0, layer 0 (pruned), embedding (twice in the code, once per order: a loop over
    // the two trunks let LICM keep weight prefetches live across both and spilled 578 VGPRs)
    auto actor = [&] {
        head_input_grad(sm, PT + kHeadT, sm.z);
        __syncthreads();
        BTR(53);
        EmbBwdPre ep;
        bwd_layer<kActorTrunk, 0, true, 36, NoHook, kBwdFull, kBwdSplit>(sm, P, PT, io.L[0], b0, &ep, io.e[0], io.xg);
        embed_bwd(sm, ep, io.epart + (size_t)blk * 2 * kEmbPart, 57);
        BTR(54);
    };
    if (actor_first) {
        actor();
        __syncthreads();  // the critic's trunk reuses every buffer
        float* dzc = sm.ctx + 64;
        for (int i = tid_x(); i < SPW * HID; i += NTHR)
            dzc[(i / HID) * LDZ + i % HID] = io.dz[1][(size_t)(b0 + i / HID) * HID + i % HID];
        __syncthreads();
    }
    if (role != 1) {  // critic: head.0, layer 1 (pruned), layer 0, embedding
        head_input_grad(sm, PT + kHeadT + D * HID, sm.ctx + 64);
        __syncthreads();
        BTR(2);
        // layer 0's LN2-backward operands are loaded at the end of layer 1's backward
        LnBwdPre l2;
        auto hook = [&] {
            ln_bwd_load(l2, io.L[1].xhat2, io.L[1].rstd2, P + kOffs.o[layer_param(kCriticTrunk, 0, N2W)], 0, b0, false);
        };
        bwd_layer<kCriticTrunk, 1, true, 4, decltype(hook), kBwdFull, kBwdSplit>(sm, P, PT + 2 * kLayerT, io.L[2], b0,
                                                                              nullptr, nullptr, nullptr, nullptr, hook);
        EmbBwdPre ep;
        bwd_layer<kCriticTrunk, 0, false, 20, NoHook, kBwdFull, kBwdSplit>(sm, P, PT + 1 * kLayerT, io.L[1], b0, &ep,
                                                                         io.e[1], io.xg, &l2);
        embed_bwd(sm, ep, io.epart + ((size_t)blk * 2 + 1) * kEmbPart);
        __syncthreads();
        BTR(52);
    }
    if (role != 2 && !actor_first) actor();
}

// ================================================================== K7: position-split training step
// Small minibatches leave most CUs idle in the 16-samples-per-workgroup kernels above (minibatch 64:
// 8 workgroups, each with ~30 MFLOP of its critic trunk = ~48 us at one CU's MFMA peak). Here every
// full (unpruned) encoder layer runs as 5 workgroups per 16-sample block, one per window position
// (16 tokens = one MFMA column tile): token-local work (embedding, Q|K|V projection, out-projection,
// LayerNorms, FFN) splits exactly; attention needs every position's K / V, so the launches are cut
// there and the K / V rows go through the workspace (L2-resident at these sizes):
//   F1  block x trunk x position: gather, embedding, layer-0 Q|K|V of the position
//   F2  block x (critic x 5 positions | actor x position 4): layer-0 attention for the position's
//       queries, out-proj + LN1 + FFN + LN2; critic: layer-1 K|V of the position (Q at position 4);
//       actor: the head
//   F3  block (critic): layer 1 (pruned: position 4) attention + tail + head, the loss partials
//   B1  block x trunk: loss / head backward, the pruned top layer's backward down to its dqkv rows
//   B2  block x trunk x position: dL/d(top layer input) at the position = W_in^T dqkv + residual;
//       actor: embedding backward; critic: layer-0 backward for the position's queries -- its dq rows
//       and its share of every position's dk / dv (kvc)
//   B3  block x position (critic): dk / dv of the position = the 5 shares in position order (fixed:
//       deterministic), W_in^T, residual, embedding backward
// Partial rows (bias / LayerNorm / embedding gradients) are per (block, position): row b * 5 + s
// (per-block layers use row b * 5). The same weight-gradient GEMM, reduction and Adam follow.
constexpr int LDQ = 3 * D + 8;  // a [dq | dk | dv] row in LDS (392 floats: 2 mod 16 slots of 16 B)

__device__ __forceinline__ void ps_mask(Smem& sm, const float* __restrict__ mask, int b0) {
    if (tid_x() < SPW * S) sm.mask[tid_x()] = mask[(size_t)b0 * S + tid_x()] != 0.f;
}

// Workspace rows [(b0 + p) * 5 + s][c0 .. c0 + cols) -> LDS rows s * 16 + p (stride lds)
__device__ __forceinline__ void ps_rows_in(float* dst, int lds, const float* __restrict__ src, int ld, int c0, int cols,
                                           int s, int b0) {
    const int n4 = cols / 4;
    for (int i = tid_x(); i < SPW * n4; i += NTHR) {
        const int p = i / n4, q = i - p * n4;
        st4(dst + (s * SPW + p) * lds + 4 * q, ld4(src + (size_t)trow(s * SPW + p, b0) * ld + c0 + 4 * q));
    }
}

// Embedding of window position s (transformer_net.py:57-59): h = relu(W_e x + b_e) + pos[s] -> sm.h
// rows 16 s + p and the e / h0 workspace rows; wave w computes features [16 w, 16 w + 16).
// The embedding's global operands (ps_embed_load: issued by k_ps_f1 before the window gather).
struct PsEmbPre {
    f32x4 a, bb, pp;
};
__device__ __forceinline__ PsEmbPre ps_embed_load(const float* __restrict__ P, int trunk, int s) {
    const float* We = P + kOffs.o[trunk + EMB_W];
    const int l = lane_id(), i16 = l & 15, g = l >> 4, wv = tid_x() >> 6;
    const int f = 16 * wv + i16;
    PsEmbPre r;
    r.a.x = 4 * g + 0 < IN ? We[f * IN + 4 * g + 0] : 0.f;
    r.a.y = 4 * g + 1 < IN ? We[f * IN + 4 * g + 1] : 0.f;
    r.a.z = 4 * g + 2 < IN ? We[f * IN + 4 * g + 2] : 0.f;
    r.a.w = 4 * g + 3 < IN ? We[f * IN + 4 * g + 3] : 0.f;
    r.bb = ld4(P + kOffs.o[trunk + EMB_B] + 16 * wv + 4 * g);
    r.pp = ld4(P + kOffs.o[trunk + POS] + s * D + 16 * wv + 4 * g);
    return r;
}
template <bool PL = false>  // PL: also the planes of h into sm.ctx (ps_inproj_split's operand)
__device__ void ps_embed(Smem& sm, const PsEmbPre& ep, float* __restrict__ e_out, float* __restrict__ h_out, int b0,
                         int s, int ti) {
    const int l = lane_id(), i16 = l & 15, g = l >> 4, wv = tid_x() >> 6;
    const f32x4 a = ep.a, bb = ep.bb, pp = ep.pp;
    const f32x4 x = ld4(sm.x + (s * SPW + i16) * LDX + 4 * g);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], x[j], acc, 0, 0, 0);
    f32x4 e = acc + bb;
    e.x = fmaxf(e.x, 0.f); e.y = fmaxf(e.y, 0.f); e.z = fmaxf(e.z, 0.f); e.w = fmaxf(e.w, 0.f);
    const f32x4 v = e + pp;
    st4(sm.h + (s * SPW + i16) * LDH + 16 * wv + 4 * g, v);
    if constexpr (PL)  // scaled per token (its window row's range)
        hsplit_store(reinterpret_cast<_Float16*>(sm.ctx), psw((s * SPW + i16), 16 * wv + 4 * g),
                     v * e_sc_v(sm.rtab[kRtE + 2 * ti], sm.rtab[kRtE + 2 * ti + 1], sm.tmax[s * SPW + i16]).sc);
    const size_t r = (size_t)trow(s * SPW + i16, b0);
    st4(e_out + r * D + 16 * wv + 4 * g, e);
    st4(h_out + r * D + 16 * wv + 4 * g, v);
}

// in_proj rows [16 tile0, 384) of the 16 tokens of position s (sm.h rows 16 s + p) -> qkv rows
// (Q = rows 0-127, K = 128-255, V = 256-383 of a [b * 5 + s][384] row), bias added.
__device__ void ps_inproj(Smem& sm, const float* __restrict__ W, const float* __restrict__ bias,
                          float* __restrict__ qkv, int tile0, int s, int b0) {
    const int l = lane_id(), i16 = l & 15, g = l >> 4, wv = tid_x() >> 6;
    const size_t r = (size_t)trow(s * SPW + i16, b0);
    for (int t = tile0 + wv; t < 3 * D / 16; t += NW) {  // wave-uniform
        const int row = 16 * t;
        const f32x4 bb = ld4(bias + row + 4 * g);
        f32x4 acc[1];
        zero(acc);
        gemm_tile<1, 4>(acc, prefetch<4>(W, D, row, 0), W, D, row, 0, sm.h, LDH, s * SPW);
        st4(qkv + r * 3 * D + row + 4 * g, acc[0] + bb);
    }
}

// ps_inproj as split products: the operand planes of the 16 tokens at X rows 16 s + p, W's split copy at soff.
// Every weight block and bias of the wave's (at most 3) row tiles is loaded in one round
// (ps_inproj_load, which a caller issues ahead of the operand's producer): one exposed L2 round trip
// instead of one per tile -- the same MFMA sequence per tile, so the same sums.
constexpr int kPsInTiles = 3;  // row tiles per wave: 24 tiles of in_proj over 8 waves
struct PsInPre {
    HPre<4> w[kPsInTiles];
    f32x4 bb[kPsInTiles];
};
__device__ __forceinline__ void ps_inproj_load(PsInPre& r, const float* __restrict__ P, int soff,
                                               const float* __restrict__ bias, int tile0) {
    const int g = lane_id() >> 4, wv = tid_x() >> 6;
#pragma unroll
    for (int k = 0; k < kPsInTiles; ++k) {
        // unconditional loads (a tile below tile0 reloads tile wv: loaded, never used)
        const int t = tile0 + wv + NW * k, row = 16 * (t < 3 * D / 16 ? t : wv);
        r.w[k] = hprefetch<4>(P, soff, D, row, 0);
        r.bb[k] = ld4(bias + row + 4 * g);
    }
}
// inv: 2^s of the operand at this lane's token (the caller's: layer 0 per token, layer 1 static)
__device__ void ps_inproj_split(const PsInPre& pre, const float* __restrict__ P, int soff, float* __restrict__ qkv,
                                int tile0, int s, int b0, const _Float16* X, float inv) {
    const int l = lane_id(), i16 = l & 15, g = l >> 4, wv = tid_x() >> 6;
    const size_t r = (size_t)trow(s * SPW + i16, b0);
#pragma unroll
    for (int k = 0; k < kPsInTiles; ++k) {
        const int t = tile0 + wv + NW * k;
        if (t >= 3 * D / 16) break;  // wave-uniform
        const int row = 16 * t;
        f32x4 hi[1], lo[1];
        zero(hi);
        zero(lo);
        hgemm_tile<1, 4>(hi, lo, pre.w[k], P, soff, D, row, 0, X, s * SPW);
        st4(qkv + r * 3 * D + row + 4 * g, (hi[0] + lo[0] * kLoScale) * inv + pre.bb[k]);
    }
}
static_assert(NW * kPsInTiles == 3 * D / 16, "ps_inproj_load covers every in_proj row tile");

// Q of position s and K | V of all five positions for the heads of chunk c -> sm.big [tok][Q|K|V];
// in two halves so that chunk 1's loads can be in flight during chunk 0's attention
constexpr int kQkvItems = SPW * 16 + TOK * 32, kQkvIt = (kQkvItems + NTHR - 1) / NTHR;
struct QkvPre {
    f32x4 v[kQkvIt];
};
__device__ __forceinline__ void ps_qkv_item(int i, int s, int& tok, int& part, int& q) {
    if (i < SPW * 16) {
        tok = s * SPW + i / 16; part = 0; q = i % 16;
    } else {
        const int k = i - SPW * 16;
        tok = k / 32; part = 1 + (k % 32) / 16; q = k % 16;
    }
}
__device__ __forceinline__ void ps_qkv_load(QkvPre& r, const float* __restrict__ qkv, int c, int s, int b0) {
#pragma unroll
    for (int k = 0; k < kQkvIt; ++k) {
        const int i = tid_x() + NTHR * k;
        if (i < kQkvItems) {
            int tok, part, q;
            ps_qkv_item(i, s, tok, part, q);
            r.v[k] = ld4(qkv + (size_t)trow(tok, b0) * 3 * D + part * D + 64 * c + 4 * q);
        }
    }
}
__device__ __forceinline__ void ps_qkv_store(Smem& sm, const QkvPre& r, int s) {
#pragma unroll
    for (int k = 0; k < kQkvIt; ++k) {
        const int i = tid_x() + NTHR * k;
        if (i < kQkvItems) {
            int tok, part, q;
            ps_qkv_item(i, s, tok, part, q);
            st4(sm.big + tok * LDB + part * 64 + 4 * q, r.v[k]);
        }
    }
}
// the attention of both chunks (K7 F2 / F3): chunk 1's Q | K | V loads overlap chunk 0's attention
// (PLANES: the output's planes scaled for layer `layer` of trunk `trunk`, P's range table)
template <bool PLANES, int trunk, int layer>
__device__ __forceinline__ void ps_attention(Smem& sm, const float* __restrict__ qkv, int s, int b0,
                                             const float* __restrict__ P) {
    QkvPre r;
    ps_qkv_load(r, qkv, 0, s, b0);
    ps_qkv_store(sm, r, s);
    __syncthreads();
    ps_qkv_load(r, qkv, 1, s, b0);
    attention_chunk<PLANES, trunk, layer>(sm, 0, s, 1, P);
    __syncthreads();
    ps_qkv_store(sm, r, s);
    __syncthreads();
    attention_chunk<PLANES, trunk, layer>(sm, 1, s, 1, P);
    __syncthreads();
}

__global__ __launch_bounds__(NTHR) void k_ps_f1(const float* __restrict__ P, const float* __restrict__ states, int B,
                                                const TrainIO io) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    const int blk = blockIdx.x / 10, r = blockIdx.x % 10, s = r % S, b0 = blk * SPW;
    const bool critic = r >= S;
    const int trunk = critic ? kCriticTrunk : kActorTrunk;
    // the actor's only layer is pruned: Q at position 4 only
    const int tile0 = critic || s == S - 1 ? 0 : D / 16;
    const int soff = critic ? split_slot(layer_param(kCriticTrunk, 0, INW)) : split_slot(layer_param(kActorTrunk, 0, INW));
    // every global operand of the embedding and of the in_proj GEMM first: their L2 round trip
    // overlaps the window gather's
    const PsEmbPre ep = ps_embed_load(P, trunk, s);
    [[maybe_unused]] PsInPre wp;
    if constexpr (kPsSplit) ps_inproj_load(wp, P, soff, P + kOffs.o[layer_param(trunk, 0, INB)], tile0);
    gather_windows<true>(sm, states, B, io, b0, r == 0, P + kRangeOff);  // one workgroup per block writes the rows
    load_rtab(sm, P);  // behind the gather's loads (its arithmetic waits on nothing they need)
    __syncthreads();
    // the step's derived scales, once: F2 / F3 and the weight-gradient GEMM read them (TrainIO::rtab_out)
    if (blockIdx.x == 0 && tid_x() < kRtN && io.rtab_out) io.rtab_out[tid_x()] = sm.rtab[tid_x()];
    ps_embed<kPsSplit>(sm, ep, io.e[critic ? 1 : 0], io.h0[critic ? 1 : 0], b0, s, critic ? 1 : 0);
    __syncthreads();
    if constexpr (kPsSplit) {
        const float m = sm.tmax[s * SPW + (lane_id() & 15)];
        ps_inproj_split(wp, P, soff, io.L[critic ? 1 : 0].qkv, tile0, s, b0, reinterpret_cast<const _Float16*>(sm.ctx),
                        critic ? e_sc<kCriticTrunk>(sm, m).inv : e_sc<kActorTrunk>(sm, m).inv);
    } else {
        ps_inproj(sm, P + kOffs.o[layer_param(trunk, 0, INW)], P + kOffs.o[layer_param(trunk, 0, INB)],
                  io.L[critic ? 1 : 0].qkv, critic || s == S - 1 ? 0 : D / 16, s, b0);
    }
}

__global__ __launch_bounds__(NTHR) void k_ps_f2(const float* __restrict__ P, const TrainIO io) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    const int blk = blockIdx.x / 6, r = blockIdx.x % 6, b0 = blk * SPW, wv = tid_x() >> 6;
    const bool critic = r < S;
    const int s = critic ? r : S - 1, ti = critic ? 1 : 0;
    // the out-projection's first weight blocks ahead of the attention (whose Q | K | V loads and
    // barriers then cover their round trip)
    [[maybe_unused]] HPre<2> po;
    if constexpr (kPsSplit)
        po = hprefetch<2>(P, critic ? split_slot(layer_param(kCriticTrunk, 0, OUTW)) : split_slot(layer_param(kActorTrunk, 0, OUTW)),
                          D, 16 * wv, 0);
    // the block's window-row maxima (F1's) first: reduced once the rows below have landed (the
    // vector memory counter retires in order), not waited for ahead of their loads
    const float a0v = a0f_load(io.tmax + (size_t)b0 * S);
    ps_mask(sm, io.mask, b0);
    ps_rows_in(sm.h, LDH, io.h0[ti], D, 0, D, s, b0);  // the layer input (residual) of the position
    load_rtab_ready(sm, io.rtab_out);  // F1's derived table, behind the loads above
    float ec[8];  // layer 0's constants (kRgE .. kRgA0 + 3 = the table's kRtE ..): uniform loads
#pragma unroll
    for (int k = 0; k < 8; ++k) ec[k] = io.rtab_out[kRtE + k];
    const float xm = a0f_finish(sm, a0v, ec, ec + 4);
    if (r == 0 && tid_x() == 0 && io.xmax) io.xmax[blk] = xm;  // the block's range for the weight gradients
    if (critic) ps_attention<kPsSplit, kCriticTrunk, 0>(sm, io.L[ti].qkv, s, b0, P);
    else ps_attention<kPsSplit, kActorTrunk, 0>(sm, io.L[ti].qkv, s, b0, P);
    [[maybe_unused]] APre<4> ph;
    if constexpr (kPsSplit) {  // the layer tails and the next in_proj as split products
        if (critic) {
            // layer 1's in_proj weights and biases are issued before LN2 (the tail's hook), behind
            // every weight load of the tail
            constexpr int s1 = split_slot(layer_param(kCriticTrunk, 1, INW));
            const int tile0 = s == S - 1 ? 0 : D / 16;
            PsInPre wp;
            auto hook = [&] { ps_inproj_load(wp, P, s1, P + kOffs.o[layer_param(kCriticTrunk, 1, INB)], tile0); };
            layer_tail_split<kCriticTrunk, 0, false, true, decltype(hook), 1>(sm, P, po, io.L[1], b0, hook, s * SPW);
            __syncthreads();
            // layer 1 (pruned) of this position: K | V, and Q at position 4, from LN2's planes in sm.h
            ps_inproj_split(wp, P, s1, io.L[2].qkv, tile0, s, b0, reinterpret_cast<const _Float16*>(sm.h),
                            op_sc<kCriticTrunk, 0, kOpLn2>(sm).inv);
            return;
        }
        auto hook = [&] {  // the head's weights before LN2
            if (wv < 4) ph = prefetch<4>(P + kOffs.o[kActorHead], D, 16 * wv, 0);
        };
        layer_tail_split<kActorTrunk, 0, true, true, decltype(hook)>(sm, P, po, io.L[0], b0, hook);
    } else {
        if (critic) {
            const APre<4> po = prefetch<4>(P + kOffs.o[layer_param(kCriticTrunk, 0, OUTW)], D, 16 * wv, 0);
            layer_tail<kCriticTrunk, 0, false, true, NoHook, 1>(sm, P, po, io.L[1], b0, NoHook{}, s * SPW);
            __syncthreads();
            // layer 1 (pruned) of this position: K | V, and Q at position 4
            ps_inproj(sm, P + kOffs.o[layer_param(kCriticTrunk, 1, INW)], P + kOffs.o[layer_param(kCriticTrunk, 1, INB)],
                      io.L[2].qkv, s == S - 1 ? 0 : D / 16, s, b0);
            return;
        }
        const APre<4> po = prefetch<4>(P + kOffs.o[layer_param(kActorTrunk, 0, OUTW)], D, 16 * wv, 0);
        layer_tail<kActorTrunk, 0, true, true>(sm, P, po, io.L[0], b0);
        if (wv < 4) ph = prefetch<4>(P + kOffs.o[kActorHead], D, 16 * wv, 0);
    }
    __syncthreads();
    head_mlp<kActorHead, 2>(sm, P, ph, sm.logits);
    store_hidden(sm, io.z[0], b0);
    if (tid_x() < SPW) {
        float* o = io.smp + (size_t)(b0 + tid_x()) * 8;
        o[5] = sm.logits[2 * tid_x()];
        o[6] = sm.logits[2 * tid_x() + 1];
    }
}

__global__ __launch_bounds__(NTHR) void k_ps_f3(const float* __restrict__ P, const TrainIO io) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    const int b0 = blockIdx.x * SPW, wv = tid_x() >> 6;
    // the out-projection's first weight blocks ahead of the attention (as k_ps_f2)
    [[maybe_unused]] HPre<2> po;
    if constexpr (kPsSplit) po = hprefetch<2>(P, split_slot(layer_param(kCriticTrunk, 1, OUTW)), D, 16 * wv, 0);
    ps_mask(sm, io.mask, b0);
    ps_rows_in(sm.h, LDH, io.L[1].h2, D, 0, D, S - 1, b0);  // layer 1's input (residual) at position 4
    load_rtab_ready(sm, io.rtab_out);  // F1's derived table, behind the loads above
    ps_attention<kPsSplit, kCriticTrunk, 1>(sm, io.L[2].qkv, S - 1, b0, P);
    APre<4> ph;
    if constexpr (kPsSplit) {  // the residual is in sm.h (ps_rows_in): PSX = 2
        auto hook = [&] {  // the head's weights before LN2
            if (wv < 4) ph = prefetch<4>(P + kOffs.o[kCriticHead], D, 16 * wv, 0);
        };
        layer_tail_split<kCriticTrunk, 1, true, true, decltype(hook), 2>(sm, P, po, io.L[2], b0, hook);
    } else {
        const APre<4> po = prefetch<4>(P + kOffs.o[layer_param(kCriticTrunk, 1, OUTW)], D, 16 * wv, 0);
        layer_tail<kCriticTrunk, 1, true, true>(sm, P, po, io.L[2], b0);
        if (wv < 4) ph = prefetch<4>(P + kOffs.o[kCriticHead], D, 16 * wv, 0);
    }
    __syncthreads();
    head_mlp<kCriticHead, 1>(sm, P, ph, sm.value);
    store_hidden(sm, io.z[1], b0);
    if (tid_x() < SPW) {  // the actor's logits (F2) beside the value: the block's loss partials
        const float* o = io.smp + (size_t)(b0 + tid_x()) * 8;
        sm.logits[2 * tid_x()] = o[5];
        sm.logits[2 * tid_x() + 1] = o[6];
    }
    __syncthreads();
    loss_partials(sm, io, b0);
}

__global__ __launch_bounds__(NTHR) void k_ps_b1(const float* __restrict__ P, const float* __restrict__ PT,
                                                const BwdIO io) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    if (tid_x() >= NTHR / 2) __builtin_amdgcn_s_setprio(1);
    const int blk = blockIdx.x >> 1, role = 1 + (blockIdx.x & 1), b0 = blk * SPW;
    ps_mask(sm, io.mask, b0);
    heads_bwd(sm, P, io, b0, role);
    __syncthreads();
    if (role == 2) {  // critic: head.0, layer 1 (pruned) down to its dqkv rows
        head_input_grad(sm, PT + kHeadT + D * HID, sm.ctx + 64);
        __syncthreads();
        bwd_layer<kCriticTrunk, 1, true, 4, NoHook, kBwdNoDx, kPsSplit>(sm, P, PT + 2 * kLayerT, io.L[2], b0, nullptr, nullptr,
                                                                 nullptr, nullptr, NoHook{}, 0, blk * S);
    } else {  // actor: head.0, layer 0 (pruned) down to its dqkv rows
        head_input_grad(sm, PT + kHeadT, sm.z);
        __syncthreads();
        bwd_layer<kActorTrunk, 0, true, 36, NoHook, kBwdNoDx, kPsSplit>(sm, P, PT, io.L[0], b0, nullptr, nullptr, nullptr,
                                                                nullptr, NoHook{}, 0, blk * S);
    }
}

// The 16 [dq | dk | dv] rows of position s -> sm.big rows p (stride LDQ); with_q = false: a pruned
// layer off its query position (dq never written there: zero)
// (kPsSplit: as the two fp16 planes of ps_dx's split products, both in one row of 2 LDQ halves,
// plane 2 at + 3 D: conflict-free ds_read_b128 like the fp32 LDQ rows)
__device__ __forceinline__ void ps_big_store(Smem& sm, int p, int q, const f32x4 v) {
    if constexpr (kPsSplit) {
        _Float16* bp = reinterpret_cast<_Float16*>(sm.big);
        f16x4 a, b;
        f16_split4(v, a, b);
        *reinterpret_cast<f16x4*>(bp + p * 2 * LDQ + 4 * q) = a;  // [p][plane 1 | plane 2 | pad]
        *reinterpret_cast<f16x4*>(bp + p * 2 * LDQ + 3 * D + 4 * q) = b;
    } else {
        st4(sm.big + p * LDQ + 4 * q, v);
    }
}
__device__ __forceinline__ void ps_dqkv_in(Smem& sm, const float* __restrict__ dqkv, bool with_q, int s, int b0) {
    for (int i = tid_x(); i < SPW * 96; i += NTHR) {
        const int p = i / 96, q = i - 96 * p;
        f32x4 v = ld4(dqkv + (size_t)trow(s * SPW + p, b0) * 3 * D + 4 * q);
        if (!with_q && q < 32) v = f32x4{0.f, 0.f, 0.f, 0.f};
        ps_big_store(sm, p, q, v);
    }
}
// dL/d(layer input) of position s = W_in^T [dq | dk | dv] (sm.big, ps_dqkv_in) + the residual rows
// res + p * res_ld (nullptr: none) -> sm.h rows 16 s + p. The split GEMM's weights (all three parts,
// every k block: ps_dx_load) are issued by the caller before the [dq | dk | dv] rows are read in, so
// their L2 round trip overlaps that one (one exposed round trip instead of one per part).
struct PsDxPre {
    HPre<4> w[3];
    f32x4 res;  // this lane's residual float4 (zero without a residual)
};
__device__ __forceinline__ void ps_dx_load(PsDxPre& r, const float* __restrict__ WinT, const float* __restrict__ res,
                                           int res_ld) {
    const int l = lane_id(), i16 = l & 15, g = l >> 4, wv = tid_x() >> 6;
#pragma unroll
    for (int part = 0; part < 3; ++part) r.w[part] = hprefetch<4>(WinT, kTSplit, 3 * D, 16 * wv, part * D);
    // unconditional (WinT's first float4 stands in when there is no residual; ps_dx then ignores it)
    r.res = ld4(res ? res + (size_t)i16 * res_ld + 16 * wv + 4 * g : WinT);
}
__device__ void ps_dx(Smem& sm, const PsDxPre& pw, const float* __restrict__ WinT, bool with_q, bool has_res,
                      int s) {
    const int l = lane_id(), i16 = l & 15, g = l >> 4, wv = tid_x() >> 6;
    const int fo = 16 * wv + 4 * g;
    f32x4 acc[1];
    zero(acc);
    if constexpr (kPsSplit) {  // WinT + kTSplit: the split copy of this layer's in_proj^T
        f32x4 lo[1];
        zero(lo);
        const _Float16* bp = reinterpret_cast<const _Float16*>(sm.big);
#pragma unroll
        for (int part = 0; part < 3; ++part) {
            if (part == 0 && !with_q) continue;
            hgemm_tile<1, 4, 4, 2 * LDQ, 3 * D>(acc, lo, pw.w[part], WinT, kTSplit, 3 * D, 16 * wv, part * D,
                                                bp + part * D, 0);
        }
        acc[0] += lo[0] * kLoScale;
    } else {
#pragma unroll
        for (int part = 0; part < 3; ++part) {
            if (part == 0 && !with_q) continue;
            gemm_tile<1, 4>(acc, prefetch<4>(WinT, 3 * D, 16 * wv, part * D), WinT, 3 * D, 16 * wv, part * D,
                            sm.big + part * D, LDQ, 0);
        }
    }
    f32x4 v = acc[0];
    if (has_res) v += pw.res;  // (wave-uniform) the residual ps_dx_load read
    st4(sm.h + (s * SPW + i16) * LDH + fo, v);
}

// Embedding backward of position s from sm.h rows 16 s + p = dL/d(h0): thread = (feature, token
// group of 4); the [pos | We | be] partial row of (block, position) -> part (only pos row s nonzero).
// Its global operands (ps_embed_bwd_load, issued by the caller ahead of the W_in^T GEMM): this
// thread's embedding values (the ReLU mask) and one float4 of the position's input rows.
struct PsEmbBwdPre {
    float ev[SPW / 4];
    f32x4 xv;
};
__device__ __forceinline__ void ps_embed_bwd_load(PsEmbBwdPre& r, const float* __restrict__ e,
                                                  const float* __restrict__ xg, int s, int b0) {
    const int f = tid_x() & (D - 1), grp = tid_x() >> 7;
    const int i = tid_x() < SPW * LDX / 4 ? tid_x() : 0;  // unconditional load (threads >= 64: unused)
    const int p = i / (LDX / 4), q = i % (LDX / 4);
    r.xv = ld4(xg + (size_t)trow(s * SPW + p, b0) * 16 + 4 * q);
#pragma unroll
    for (int k = 0; k < SPW / 4; ++k) r.ev[k] = e[(size_t)trow(s * SPW + grp + 4 * k, b0) * D + f];
}
__device__ void ps_embed_bwd(Smem& sm, const PsEmbBwdPre& r, float* __restrict__ part, int s) {
    const int f = tid_x() & (D - 1), grp = tid_x() >> 7;
    if (tid_x() < SPW * LDX / 4) {
        const int p = tid_x() / (LDX / 4), q = tid_x() % (LDX / 4);
        st4(sm.x + p * LDX + 4 * q, r.xv);
    }
    float ev[SPW / 4];
#pragma unroll
    for (int i = 0; i < SPW / 4; ++i) ev[i] = r.ev[i];
    __syncthreads();
    float acc[IN + 1], accp = 0.f;
#pragma unroll
    for (int v = 0; v < IN + 1; ++v) acc[v] = 0.f;
#pragma unroll
    for (int i = 0; i < SPW / 4; ++i) {
        const int p = grp + 4 * i;
        const float gv = sm.h[(s * SPW + p) * LDH + f];
        accp += gv;
        const float gp = ev[i] > 0.f ? gv : 0.f;
        acc[IN] += gp;
#pragma unroll
        for (int q = 0; q < LDX / 4; ++q) {
            const f32x4 x4 = ld4(sm.x + p * LDX + 4 * q);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (4 * q + k < IN) acc[4 * q + k] += gp * x4[k];
        }
    }
    constexpr int NV = IN + 1 + S;  // 20
#pragma unroll
    for (int v = 0; v < NV; ++v)
        sm.big[(grp * NV + v) * D + f] = v <= IN ? acc[v] : (v == IN + 1 + s ? accp : 0.f);
    __syncthreads();
    for (int o = tid_x(); o < NV * D; o += NTHR) {
        const int v = o >> 7, ff = o & (D - 1);
        const float sum = (sm.big[v * D + ff] + sm.big[(NV + v) * D + ff]) +
                          (sm.big[(2 * NV + v) * D + ff] + sm.big[(3 * NV + v) * D + ff]);
        const int dst = v < IN ? S * D + ff * IN + v : (v == IN ? S * D + D * IN + ff : (v - IN - 1) * D + ff);
        part[dst] = sum;
    }
}

__global__ __launch_bounds__(NTHR) void k_ps_b2(const float* __restrict__ P, const float* __restrict__ PT,
                                                const BwdIO io, float* __restrict__ kvc) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    if (tid_x() >= NTHR / 2) __builtin_amdgcn_s_setprio(1);
    const int blk = blockIdx.x / 10, r = blockIdx.x % 10, s = r % S, b0 = blk * SPW, prow = blk * S + s;
    const bool critic = r >= S, q4 = s == S - 1;
    // dL/d(input of the trunk's top, pruned layer) at position s; its residual path (LN1's input
    // gradient, compact [b] rows) exists at the query position 4 only
    const BwdLayerIO& top = io.L[critic ? 2 : 0];
    const float* WinT = PT + (critic ? 2 : 0) * kLayerT + kTWin;
    ps_mask(sm, io.mask, b0);
    ps_dqkv_in(sm, top.dqkv, q4, s, b0);
    __syncthreads();
    // (the GEMM's operands loaded here, not ahead of the dq | dk | dv rows: ahead measured 0.2-0.3 us
    // slower in this kernel, r04x)
    PsDxPre pw;
    ps_dx_load(pw, WinT, q4 ? top.dz1 + (size_t)b0 * D : nullptr, D);
    if (!critic) {  // the actor: the embedding backward's operands ahead of the GEMM
        PsEmbBwdPre eb;
        ps_embed_bwd_load(eb, io.e[0], io.xg, s, b0);
        ps_dx(sm, pw, WinT, q4, q4, s);
        __syncthreads();
        ps_embed_bwd(sm, eb, io.epart + (size_t)prow * 2 * kEmbPart, s);
        return;
    }
    ps_dx(sm, pw, WinT, q4, q4, s);
    __syncthreads();
    bwd_layer<kCriticTrunk, 0, false, 20, NoHook, kBwdPos, kPsSplit>(sm, P, PT + kLayerT, io.L[1], b0, nullptr, nullptr, nullptr,
                                                              nullptr, NoHook{}, s * SPW, prow, kvc);
}

__global__ __launch_bounds__(NTHR) void k_ps_b3(const float* __restrict__ PT, const BwdIO io,
                                                const float* __restrict__ kvc) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    const int blk = blockIdx.x / S, j = blockIdx.x % S, b0 = blk * SPW, prow = blk * S + j;
    // [dq | dk | dv] rows of position j: dq from B2 (position j), dk / dv = the five query
    // positions' shares summed in position order (deterministic); dk / dv -> the dqkv rows
    float* dqkv = io.L[1].dqkv;
    // + LN1's input gradient of layer 0 at position j (the residual path); the GEMM's weights, the
    // residual rows and the embedding backward's operands are loaded ahead of the [dq | dk | dv] rows
    const float* WinT = PT + kLayerT + kTWin;
    PsDxPre pw;
    ps_dx_load(pw, WinT, io.L[1].dz1 + (size_t)trow(j * SPW, b0) * D, S * D);
    PsEmbBwdPre eb;
    ps_embed_bwd_load(eb, io.e[1], io.xg, j, b0);
    for (int i = tid_x(); i < SPW * 96; i += NTHR) {
        const int p = i / 96, q = i - 96 * p, tok = j * SPW + p;
        const size_t row = (size_t)trow(tok, b0);
        f32x4 v;
        if (q < 32) {
            v = ld4(dqkv + row * 3 * D + 4 * q);
        } else {
            v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < S; ++s) v += ld4(kvc + ((size_t)(blk * S + s) * TOK + tok) * 2 * D + 4 * (q - 32));
            st4(dqkv + row * 3 * D + 4 * q, v);
        }
        ps_big_store(sm, p, q, v);
    }
    __syncthreads();
    ps_dx(sm, pw, WinT, true, true, j);
    __syncthreads();
    ps_embed_bwd(sm, eb, io.epart + ((size_t)prow * 2 + 1) * kEmbPart, j);
}


}  // namespace pol
}  // namespace uavhip

using namespace uavhip;

namespace uavhip {
namespace pol {
int policy_forward_train(const float* packed, const float* states, const TrainIO& io, int Bm, hipStream_t st) {
    hipLaunchKernelGGL(k_policy_forward<true>, dim3((io.split ? 2 : 1) * (Bm / SPW)), dim3(NTHR), 0, st, packed,
                       states, Bm, nullptr, 0ull, 0ull, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, io,
                       RowIO{}, uavhip_env{}, EnvOut{});
    return check_launch("k_policy_forward<train>");
}

int policy_loss_partials(const TrainIO& io, int Bm, hipStream_t st) {
    hipLaunchKernelGGL(k_loss_partials, dim3(Bm / SPW), dim3(64), 0, st, io);
    return check_launch("k_loss_partials");
}

int policy_forward_ps(const float* packed, const float* states, const TrainIO& io, int Bm, hipStream_t st) {
    const int nblk = Bm / SPW;
    hipLaunchKernelGGL(k_ps_f1, dim3(nblk * 10), dim3(NTHR), 0, st, packed, states, Bm, io);
    if (const int rc = check_launch("k_ps_f1")) return rc;
    hipLaunchKernelGGL(k_ps_f2, dim3(nblk * 6), dim3(NTHR), 0, st, packed, io);
    if (const int rc = check_launch("k_ps_f2")) return rc;
    hipLaunchKernelGGL(k_ps_f3, dim3(nblk), dim3(NTHR), 0, st, packed, io);
    return check_launch("k_ps_f3");
}

int policy_backward_ps(const float* packed, const float* packedT, const BwdIO& io, float* kvc, int Bm, hipStream_t st) {
    const int nblk = Bm / SPW;
    hipLaunchKernelGGL(k_ps_b1, dim3(nblk * 2), dim3(NTHR), 0, st, packed, packedT, io);
    if (const int rc = check_launch("k_ps_b1")) return rc;
    hipLaunchKernelGGL(k_ps_b2, dim3(nblk * 10), dim3(NTHR), 0, st, packed, packedT, io, kvc);
    if (const int rc = check_launch("k_ps_b2")) return rc;
    hipLaunchKernelGGL(k_ps_b3, dim3(nblk * S), dim3(NTHR), 0, st, packedT, io, static_cast<const float*>(kvc));
    return check_launch("k_ps_b3");
}

int policy_backward_train(const float* packed, const float* packedT, const BwdIO& io, int Bm, hipStream_t st) {
    hipLaunchKernelGGL(k_policy_backward, dim3((io.split ? 2 : 1) * (Bm / SPW)), dim3(NTHR), 0, st, packed, packedT,
                       io);
    return check_launch("k_policy_backward");
}


// flat (state_dict order, plain layout) -> packed (GEMM weights in MFMA fragment order) and, when
// packedT is given, the backward's transposed copies: per layer [in_proj^T | out_proj^T |
// linear1^T | linear2^T], then head.0^T of both heads, with packedT[((r/16) * K/16 + k/16) * 256 +
// (r%16 + 16 ((k%16)/4)) * 4 + k%4] = W[k][r]. One thread per output float4.
__global__ __launch_bounds__(256) void k_policy_pack(const float* __restrict__ flat, float* __restrict__ packed,
                                                     float* __restrict__ packedT) {
    constexpr int nq = kOffs.o[kNumParams] / 4;
    const int i = blockIdx.x * 256 + tid_x();
    if (i < nq) {
        const int f = 4 * i;
        int lo = 0, hi = kNumParams;  // parameter q: kOffs.o[q] <= f < kOffs.o[q + 1]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (f >= kOffs.o[mid]) lo = mid;
            else hi = mid;
        }
        const int local = f - kOffs.o[lo], K = kTileK[lo];
        int src = f;
        if (K != 0 && local < kSizes[lo]) {  // fragment order of [R][K]: float4 = 4 consecutive k
            const int lane = (local >> 2) & 63, blk = local >> 8, KB = K / 16;
            const int kb = blk % KB, rt = blk / KB;
            src = kOffs.o[lo] + (16 * rt + (lane & 15)) * K + 16 * kb + 4 * (lane >> 4);
        }
        // the training pack (packedT given): the split-copy weights' fp32 copies are never read
        const bool dead = !kTrainF32LayerCopies && packedT && K != 0 && split_slot(lo) >= 0;
        *reinterpret_cast<f32x4*>(packed + f) =
            dead ? f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")}
                 : *reinterpret_cast<const f32x4*>(flat + src);
        return;
    }
    if (!packedT || i >= nq + kPackedTFloats / 4) return;
    if (!kTrainF32LayerCopies && 4 * (i - nq) < kHeadT) {  // a layer weight's fp32 transposed copy: dead
        *reinterpret_cast<f32x4*>(packedT + 4 * (i - nq)) =
            f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
        return;
    }
    const int idx = 4 * (i - nq);
    int src, m, Rt, Kt;
    if (idx < kHeadT) {
        const int li = idx / kLayerT, loc = idx - li * kLayerT;
        const int trunk = li == 0 ? kActorTrunk : kCriticTrunk, layer = li == 2 ? 1 : 0;
        int which, base;
        if (loc < kTWo) { which = INW; base = kTWin; Rt = D; Kt = 3 * D; }
        else if (loc < kTW1) { which = OUTW; base = kTWo; Rt = D; Kt = D; }
        else if (loc < kTW2) { which = L1W; base = kTW1; Rt = D; Kt = FF; }
        else { which = L2W; base = kTW2; Rt = FF; Kt = D; }
        src = kOffs.o[layer_param(trunk, layer, which)];
        m = loc - base;
    } else {  // head.0 weight [64][128] of the actor / critic head, transposed
        const int h = (idx - kHeadT) / (D * HID);
        src = kOffs.o[h ? kCriticHead : kActorHead];
        m = idx - kHeadT - h * D * HID;
        Rt = D;
        Kt = HID;
    }
    const int lane = (m >> 2) & 63, blk = m >> 8, KBt = Kt / 16;
    const int kb = blk % KBt, rt = blk / KBt;
    const int r = 16 * rt + (lane & 15), k = 16 * kb + 4 * (lane >> 4);
    const float* w = flat + src + r;
    *reinterpret_cast<f32x4*>(packedT + idx) = f32x4{w[k * Rt], w[(k + 1) * Rt], w[(k + 2) * Rt], w[(k + 3) * Rt]};
}

// flat -> the split copies of the kSplitParam weights (policy_layout.hpp): one thread per lane of a
// (16-row tile, 32-k block), two f16x8 stores (w1 = f16(w), w2 = f16((w - w1) 2^11), round to nearest).
__global__ __launch_bounds__(256) void k_policy_split(const float* __restrict__ flat, float* __restrict__ packed) {
    const int i = blockIdx.x * 256 + tid_x();
    if (i < kRangeFloats) packed[kRangeOff + i] = 0.f;  // the range table, ahead of k_policy_range's maxima
    int si = 0, base = 0;
    while (si < kNumSplit && i >= base + kSizes[kSplitParam[si]] / 8) base += kSizes[kSplitParam[si++]] / 8;
    if (si >= kNumSplit) return;
    const int q = kSplitParam[si], K = kTileK[q], u = i - base;  // u = (t * K/32 + kb) * 64 + lane
    const int l = u & 63, blk = u >> 6, kb = blk % (K / 32), t = blk / (K / 32);
    const float* src = flat + kOffs.o[q] + (size_t)(16 * t + (l & 15)) * K + 32 * kb + 8 * (l >> 4);
    const f32x4 a = *reinterpret_cast<const f32x4*>(src), b = *reinterpret_cast<const f32x4*>(src + 4);
    f16x8 w1, w2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float w = j < 4 ? a[j] : b[j - 4];
        w1[j] = (_Float16)w;
        w2[j] = f16_lo(w, w1[j]);
    }
    f16x8* dst = reinterpret_cast<f16x8*>(packed + kSplitOffs.o[si]) + (size_t)blk * 128 + l;
    dst[0] = w1;
    dst[64] = w2;
}

// The range table (policy_layout.hpp) of the flat parameters: kRangeSlices blocks per parameter,
// each an atomic max of its slice's max |param| on the float bits into the parameter's slot (zeroed
// by k_policy_split; non-negative floats order like their bits). One block per parameter looped
// over up to 49 k floats: 28 us per pack.
constexpr int kRangeSlices = 8;
__global__ __launch_bounds__(256) void k_policy_range(const float* __restrict__ flat, float* __restrict__ packed) {
    __shared__ float red[4];
    const int q = blockIdx.x / kRangeSlices, sl = blockIdx.x % kRangeSlices;
    const int n = kSizes[q], per = (n + kRangeSlices - 1) / kRangeSlices, i0 = sl * per, i1 = min(n, i0 + per);
    float m = 0.f;
    for (int i = i0 + tid_x(); i < i1; i += 256) m = fmaxf(m, fabsf(flat[kOffs.o[q] + i]));
    m = wave_max(m);
    if (lane_id() == 0) red[tid_x() >> 6] = m;
    __syncthreads();
    if (tid_x() == 0)
        atomicMax(reinterpret_cast<unsigned*>(packed + kRangeOff + kRgMax + q),
                  __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

int policy_split(const float* flat, float* packed, hipStream_t st) {
    constexpr int n = (kRangeOff - kOffs.o[kNumParams]) / 8;
    hipLaunchKernelGGL(k_policy_split, dim3((n + 255) / 256), dim3(256), 0, st, flat, packed);
    if (const int rc = check_launch("k_policy_split")) return rc;
    hipLaunchKernelGGL(k_policy_range, dim3(kNumParams * kRangeSlices), dim3(256), 0, st, flat, packed);
    return check_launch("k_policy_range");
}

// flat -> the split copies of the three layers' transposed weights (packedT + kTSplit): one thread
// per lane of a (16-row tile, 32-k block) of W^T, W^T[r][k] = W[k][r] gathered from the flat rows.
__global__ __launch_bounds__(256) void k_policyT_split(const float* __restrict__ flat, float* __restrict__ packedT) {
    const int i = blockIdx.x * 256 + tid_x();  // lane index over all 3 x kLayerT / 8 (tile, block, lane)
    if (i >= kHeadT / 8) return;
    const int li = i / (kLayerT / 8), loc = i - li * (kLayerT / 8);
    const int trunk = li == 0 ? kActorTrunk : kCriticTrunk, layer = li == 2 ? 1 : 0;
    int which, base, Rt, Kt;  // W^T is [Rt][Kt]; W flat [Kt][Rt]
    if (loc < kTWo / 8) { which = INW; base = kTWin; Rt = D; Kt = 3 * D; }
    else if (loc < kTW1 / 8) { which = OUTW; base = kTWo; Rt = D; Kt = D; }
    else if (loc < kTW2 / 8) { which = L1W; base = kTW1; Rt = D; Kt = FF; }
    else { which = L2W; base = kTW2; Rt = FF; Kt = D; }
    const int u = loc - base / 8, l = u & 63, blk = u >> 6, kb = blk % (Kt / 32), rt = blk / (Kt / 32);
    const int r = 16 * rt + (l & 15), k0 = 32 * kb + 8 * (l >> 4);
    const float* w = flat + kOffs.o[layer_param(trunk, layer, which)] + r;
    f16x8 w1, w2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = w[(size_t)(k0 + j) * Rt];
        w1[j] = (_Float16)v;
        w2[j] = f16_lo(v, w1[j]);
    }
    f16x8* dst = reinterpret_cast<f16x8*>(packedT + kTSplit + li * kLayerT + base) + (size_t)blk * 128 + l;
    dst[0] = w1;
    dst[64] = w2;
}

int policy_pack_train(const float* flat, float* packed, float* packedT, hipStream_t st) {
    const int items = kOffs.o[kNumParams] / 4 + kPackedTFloats / 4;
    hipLaunchKernelGGL(k_policy_pack, dim3((items + 255) / 256), dim3(256), 0, st, flat, packed, packedT);
    if (const int rc = check_launch("k_policy_pack")) return rc;
    hipLaunchKernelGGL(k_policyT_split, dim3((kHeadT / 8 + 255) / 256), dim3(256), 0, st, flat, packedT);
    if (const int rc = check_launch("k_policyT_split")) return rc;
    return policy_split(flat, packed, st);
}
}  // namespace pol
}  // namespace uavhip

extern "C" int uavhip_policy_pack(const float* flat, float* packed, uavhip_stream_t stream) {
    if (!flat || !packed) {
        set_error("uavhip_policy_pack: NULL pointer");
        return UAVHIP_EINVAL;
    }
    const int n = pol::kOffs.o[pol::kNumParams] / 4;
    hipLaunchKernelGGL(pol::k_policy_pack, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, flat, packed,
                       nullptr);
    if (const int rc = check_launch("k_policy_pack")) return rc;
    return pol::policy_split(flat, packed, (hipStream_t)stream);
}

extern "C" int32_t uavhip_policy_layout(int32_t* offsets, int32_t max_offsets) {
    if (offsets)
        for (int i = 0; i < pol::kNumParams && i < max_offsets; ++i) offsets[i] = pol::kOffs.o[i];
    return pol::kOffs.o[pol::kNumParams];
}

extern "C" int32_t uavhip_policy_split_layout(int32_t* params, int32_t* offsets, int32_t max_entries) {
    for (int i = 0; i < pol::kNumSplit && i < max_entries; ++i) {
        if (params) params[i] = pol::kSplitParam[i];
        if (offsets) offsets[i] = pol::kSplitOffs.o[i];
    }
    return pol::kPackedFloats;
}

extern "C" int32_t uavhip_policy_range_table(const float* max_abs, float* table) {
    if (!max_abs || !table) return pol::kRangeFloats;
    float t[pol::kRangeFloats] = {};
    for (int q = 0; q < pol::kNumParams; ++q) t[pol::kRgMax + q] = max_abs[q];
    pol::range_derive(t);
    for (int k = 0; k < pol::kRangeFloats; ++k) table[k] = t[k];
    return pol::kRangeFloats;
}

extern "C" int32_t uavhip_policy_tiling(int32_t* kcols, int32_t max_params) {
    if (kcols)
        for (int i = 0; i < pol::kNumParams && i < max_params; ++i) kcols[i] = pol::kTileK[i];
    return pol::kNumParams;
}

#ifdef UAVHIP_POLICY_TRACE
extern "C" int uavhip_policy_trace(unsigned long long* out, int n) {
    const int total = 256 * 2 * pol::kTraceSlots;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pol::g_ptrace), sizeof(unsigned long long) * (n < total ? n : total), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int uavhip_policy_btrace(unsigned long long* out, int n) {  // k_policy_backward stamps
    const int total = 256 * 2 * pol::kTraceSlots;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pol::g_btrace), sizeof(unsigned long long) * (n < total ? n : total), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

static int check_policy(const char* fn, const uavhip_policy* policy, const float* states, int32_t B) {
    if (!policy || !policy->weights || !states || B <= 0) {
        set_error("%s: NULL policy/weights/states or B=%d", fn, B);
        return UAVHIP_EINVAL;
    }
    if (policy->n_floats != pol::kPackedFloats || policy->d_model != pol::D || policy->n_heads != pol::NH ||
        policy->d_ff != pol::FF || policy->d_head_hidden != pol::HID || policy->actor_layers != 1 ||
        policy->critic_layers != 2) {
        set_error("%s: unsupported architecture / packed size %d (expected %d)", fn, policy->n_floats,
                  pol::kPackedFloats);
        return UAVHIP_EINVAL;
    }
    return UAVHIP_OK;
}

extern "C" int uavhip_policy_forward(const uavhip_policy* policy, const float* states, int32_t B,
                                     const int8_t* actions_in, uint64_t seed, uint64_t offset,
                                     const uint64_t* offset_dev, int8_t* action_out, float* logp, float* value,
                                     float* entropy, float* logits, uavhip_stream_t stream) {
    if (const int rc = check_policy("uavhip_policy_forward", policy, states, B)) return rc;
    const int grid = (B + pol::SPW - 1) / pol::SPW;
    hipLaunchKernelGGL(pol::k_policy_forward<false>, dim3(grid), dim3(pol::NTHR), 0, (hipStream_t)stream,
                       policy->weights, states, (int)B, actions_in, seed, offset, offset_dev, action_out, logp, value,
                       entropy, logits, pol::TrainIO{}, pol::RowIO{}, uavhip_env{}, pol::EnvOut{});
    return check_launch("k_policy_forward");
}

extern "C" int64_t uavhip_policy_rowproj_floats(int32_t B) {
    return B > 0 ? pol::kPposFloats + (int64_t)pol::S * B * pol::kRowFloats : -1;
}

extern "C" int uavhip_policy_forward_rows(const uavhip_policy* policy, const float* states, int32_t B,
                                          float* rowproj, int32_t step, int32_t fill, const int8_t* actions_in,
                                          uint64_t seed, uint64_t offset, const uint64_t* offset_dev,
                                          int8_t* action_out, float* logp, float* value, float* entropy,
                                          float* logits, uavhip_stream_t stream) {
    if (const int rc = check_policy("uavhip_policy_forward_rows", policy, states, B)) return rc;
    if (!rowproj || step < 0 || (int64_t)B * pol::S * pol::kRowFloats >= (int64_t)1 << 31) {
        set_error("uavhip_policy_forward_rows: NULL rowproj, step=%d < 0 or B=%d above the ring's 32-bit offsets",
                  step, B);
        return UAVHIP_EINVAL;
    }
    const int grid = (B + pol::SPW - 1) / pol::SPW;
    const pol::RowIO rio{rowproj, (int)B, (int)step};
    if (fill) {
        hipLaunchKernelGGL(pol::k_policy_rows_fill, dim3(grid > pol::kPposParts ? grid : pol::kPposParts), dim3(pol::NTHR), 0,
                           (hipStream_t)stream,
                           policy->weights, states, rio);
        if (const int rc = check_launch("k_policy_rows_fill")) return rc;
    }
    hipLaunchKernelGGL((pol::k_policy_forward<false, true>), dim3(grid), dim3(pol::NTHR), 0, (hipStream_t)stream,
                       policy->weights, states, (int)B, actions_in, seed, offset, offset_dev, action_out, logp, value,
                       entropy, logits, pol::TrainIO{}, rio, uavhip_env{}, pol::EnvOut{});
    return check_launch("k_policy_forward_rows");
}

// Value-only ring forward (the rollout's bootstrap V(s_T)): the critic trunk and head of
// uavhip_policy_forward_rows, bitwise its value output; the actor's ring row is not written.
extern "C" int uavhip_policy_value_rows(const uavhip_policy* policy, const float* states, int32_t B, float* rowproj,
                                        int32_t step, int32_t fill, float* value, uavhip_stream_t stream) {
    if (const int rc = check_policy("uavhip_policy_value_rows", policy, states, B)) return rc;
    if (!rowproj || !value || step < 0 || (int64_t)B * pol::S * pol::kRowFloats >= (int64_t)1 << 31) {
        set_error("uavhip_policy_value_rows: NULL rowproj / value, step=%d < 0 or B=%d above the ring's 32-bit offsets",
                  step, B);
        return UAVHIP_EINVAL;
    }
    const int grid = (B + pol::SPW - 1) / pol::SPW;
    const pol::RowIO rio{rowproj, (int)B, (int)step};
    if (fill) {
        hipLaunchKernelGGL(pol::k_policy_rows_fill, dim3(grid > pol::kPposParts ? grid : pol::kPposParts), dim3(pol::NTHR), 0,
                           (hipStream_t)stream, policy->weights, states, rio);
        if (const int rc = check_launch("k_policy_rows_fill")) return rc;
    }
    hipLaunchKernelGGL((pol::k_policy_forward<false, true, 0, true>), dim3(grid), dim3(pol::NTHR), 0, (hipStream_t)stream,
                       policy->weights, states, (int)B, nullptr, 0ull, 0ull, nullptr, nullptr, nullptr, value, nullptr,
                       nullptr, pol::TrainIO{}, rio, uavhip_env{}, pol::EnvOut{});
    return check_launch("k_policy_value_rows");
}

// Fused rollout step: uavhip_policy_forward_rows (sampling) + uavhip_env_step (T = 1) of env e
// on window b = e, one launch. N, M <= 64 (one env per wave); B = env->E.
extern "C" int uavhip_rollout_step(const uavhip_policy* policy, const uavhip_env* env, const float* states,
                                   float* rowproj, int32_t step, int32_t fill, uint64_t seed, uint64_t offset,
                                   const uint64_t* offset_dev, int8_t* action_out, float* logp, float* value,
                                   int32_t auto_reset, float* obs_out, double* reward, uint8_t* done, double* info,
                                   uavhip_stream_t stream) {
    if (const int rc = validate_env(env, true)) return rc;
    const int32_t B = env->E;
    if (const int rc = check_policy("uavhip_rollout_step", policy, states, B)) return rc;
    if (env->N > 64 || env->M > 64 || !action_out || !obs_out || !reward || !done) {
        set_error("uavhip_rollout_step: N=%d, M=%d must be <= 64 and action/obs/reward/done non-NULL", env->N, env->M);
        return UAVHIP_EINVAL;
    }
    if (!rowproj || step < 0 || (int64_t)B * pol::S * pol::kRowFloats >= (int64_t)1 << 31) {
        set_error("uavhip_rollout_step: NULL rowproj, step=%d < 0 or E=%d above the ring's 32-bit offsets", step, B);
        return UAVHIP_EINVAL;
    }
    const int grid = (B + pol::SPW - 1) / pol::SPW;
    const pol::RowIO rio{rowproj, (int)B, (int)step};
    if (fill) {
        hipLaunchKernelGGL(pol::k_policy_rows_fill, dim3(grid > pol::kPposParts ? grid : pol::kPposParts), dim3(pol::NTHR), 0,
                           (hipStream_t)stream,
                           policy->weights, states, rio);
        if (const int rc = check_launch("k_policy_rows_fill")) return rc;
    }
    hipLaunchKernelGGL((pol::k_policy_forward<false, true, pol::kEnvBoth>), dim3(grid), dim3(pol::NTHR), 0, (hipStream_t)stream,
                       policy->weights, states, (int)B, nullptr, seed, offset, offset_dev, action_out, logp, value,
                       nullptr, nullptr, pol::TrainIO{}, rio, *env,
                       pol::EnvOut{(int)auto_reset, obs_out, reward, done, info});
    return check_launch("k_rollout_step");
}

extern "C" int uavhip_rollout_steps(const uavhip_policy* policy, const uavhip_env* env, float* obs, float* rowproj,
                                    int32_t step, int32_t n, int32_t fill, uint64_t seed, uint64_t offset,
                                    uint64_t offset_stride, const uint64_t* offset_dev, int8_t* actions, float* logp,
                                    float* value, int32_t auto_reset, double* reward, uint8_t* done, double* info,
                                    uavhip_stream_t stream) {
    if (const int rc = validate_env(env, true)) return rc;
    const int32_t B = env->E;
    if (const int rc = check_policy("uavhip_rollout_steps", policy, obs, B)) return rc;
    if (env->N > 64 || env->M > 64 || (env->flags & UAVHIP_ENV_OBS_F16) || !actions || !logp || !value || !reward ||
        !done || n <= 0) {
        set_error("uavhip_rollout_steps: N=%d, M=%d must be <= 64, observations f32, n=%d > 0 and "
                  "actions/logp/value/reward/done non-NULL", env->N, env->M, n);
        return UAVHIP_EINVAL;
    }
    if (!rowproj || step < 0 || (int64_t)B * pol::S * pol::kRowFloats >= (int64_t)1 << 31) {
        set_error("uavhip_rollout_steps: NULL rowproj, step=%d < 0 or E=%d above the ring's 32-bit offsets", step, B);
        return UAVHIP_EINVAL;
    }
    const int grid = (B + pol::SPW - 1) / pol::SPW;
    const pol::RowIO rio{rowproj, (int)B, (int)step};
    if (fill) {
        hipLaunchKernelGGL(pol::k_policy_rows_fill, dim3(grid > pol::kPposParts ? grid : pol::kPposParts), dim3(pol::NTHR), 0,
                           (hipStream_t)stream,
                           policy->weights, obs, rio);
        if (const int rc = check_launch("k_policy_rows_fill")) return rc;
    }
    const long long stride = (long long)B * pol::S * pol::IN;
    return pol::launch_rollout_steps(policy->weights, obs, (int)B, seed, offset, offset_dev, actions, logp, value, rio,
                                     *env, pol::EnvOut{(int)auto_reset, obs + stride, reward, done, info},
                                     pol::StepSeq{(int)n, stride, offset_stride}, (hipStream_t)stream);
}
#else   // the steps TU ends after k_rollout_steps
}  // namespace pol
}  // namespace uavhip
#endif  // !UAVHIP_STEPS_TU
