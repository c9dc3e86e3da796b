// Fused field-MLP forward: every Linear (+ bias + ReLU) of a NerfModel in ONE launch
// (a7, barf/model_interpolation_architecture.py:96-141; contract in include/nerf_amd.h).
//
// Layer-by-layer GEMMs move each 256-wide fp32 activation through HBM twice (written by
// one launch, read by the next: 536 MB per layer at 262 144 samples).  Here a wave owns 16 samples
// (8 waves, two per SIMD) and keeps their layer input in registers across the whole network:
//
//   out^T[n][s] = W[n][:] . x^T[:][s]    A operand = weights (rows n), B = activations (cols s)
//
// on v_mfma_f32_16x16x32_bf16.  Its 16x16 accumulator holds, in lane (s, g) (s = lane & 15,
// g = lane >> 4), output rows 4g .. 4g+3 of sample s.  Output rows 32q .. 32q+15 and 32q+16 ..
// 32q+31 give lane (s, g) exactly the eight k-values it must supply as the B operand of k-block q
// of the next layer, once the reduction index is permuted the same way in the packed weights
// (element j of lane group g <-> feature 32q + 16(j >> 2) + 4g + (j & 3)).  bias + ReLU + the bf16
// hi/lo split (3 x bf16 products, as linear_x3.hip) are applied in registers.
//
// A chunk is 16 output rows: its MFMA steps interleave the previous chunk's epilogue (bias, ReLU,
// fp32 stores, mask bits, hi/lo split) in four parts, whose split halves go to the wave's
// 16 KB LDS image of the next layer's operand; at the end of the layer that image is read
// back into the operand registers (compile-time indices: no register array is ever indexed at run
// time).  MODE_DGRAD runs the backward's input-gradient chain with the same loop: W^T images, the
// forward's ReLU bits applied to each incoming gradient row, dY of every layer stored.
//
// Weights (2.6 MB for NerfModel) stream through LDS: the register-fed k-blocks of a chunk
// ([kb][hi 1 KB | lo 1 KB], lane-linear 16 B per lane: one conflict-free ds_read_b128 each) are
// LDS-DMA'd (buffer-addressed) into a 2 x 16 KB ring one chunk ahead and shared by the waves, so
// the weights cross L2 -> LDS once per 128 samples.  The k-blocks fed by HBM inputs (encodings,
// or the head / density gradients of the backward chain) and the biases are read by each wave
// from L2.  LDS: 32 KB ring + 8 x 16 KB operand images = 160 KB.  Only HBM-fed inputs are loaded
// and only what the backward needs (each layer's output, its ReLU mask bits, the density column)
// is stored; waits are counted (asm fragment reads, a per-layer DMA table in VGPRs) so the
// prefetch is never drained.
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "common.h"
#include "encode_common.h"
#include "composite_common.h"
#include "hashgrid_common.h"

using namespace nerf;

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

constexpr int SLOT_BYTES = 16 * 1024;      // register-fed part of a 16-row chunk: <= 8 k-blocks x 2 KB
constexpr int NSLOT = 2;
constexpr int SB = 1;                      // 16-sample column blocks per wave
constexpr int XIMG_BYTES = SB * 16 * 1024; // per wave: the next layer's operand, [kb][sb][hi|lo][lane] 16 B
constexpr int WG = 512 / SB;               // 8 waves (two per SIMD) of 16 samples
constexpr int NWAVE = WG / 64;
constexpr int SPW = 16 * SB;               // samples per wave
constexpr int TILE = NWAVE * SPW;          // samples per workgroup tile
constexpr int KBMAX = 8;                   // register-fed 32-deep k-blocks (256 features)
constexpr unsigned OOB = 0x80000000u;      // buffer offset past every num_records: load 0 / drop store
constexpr int RSRC_W3 = 0x00020000;
// cache policy of the layer-output stores: nontemporal (aux bit 1, `nt`).  The outputs are written
// once and read back only by the weight-gradient launches (they do not fit the caches anyway), and
// every counted wait for a chunk's weight DMA also waits for the stores issued before it; with
// the default policy those stores held the forward at 4.56 ms per mip step, nontemporal 3.49 ms
// (the input-gradient chain 4.39 -> 3.74), results bitwise unchanged
constexpr int ST_AUX = 2;
// vector-memory ops issued after a chunk's DMA (at the start of its predecessor) before the chunk
// starts: the predecessor's 2 epilogue stores (absent outputs included, as dropped stores) and, in
// the forward, the bias load at the start of the chunk itself.  The input-gradient chain has no
// biases and loads none: a zero-bias load there, waited for at the epilogue, made every chunk wait
// for the previous chunk's dY stores (profiles/r05ac).
// kernel modes: bit 0 = the backward's input-gradient chain (else the forward), bit 1 = one bf16
// pass (hi * hi: matmul precision "medium", the reference's single-pass bf16 / fp16 products) instead
// of the 3 x bf16 split (lo * hi + hi * lo + hi * hi: "high")
constexpr bool is_fwd(int mode) { return (mode & 1) == 0; }
constexpr bool is_x1(int mode) { return (mode & 2) != 0; }
template <int MODE>
constexpr int after_dma_vm() { return is_fwd(MODE) ? 1 + 2 * SB : 2 * SB; }
// Layer-output stores in chunk pairs: a 16-row chunk is 64 B of each sample row, half a 128-B line.
// The even chunk's values wait in registers for the odd one's.  The input-gradient chain writes each
// pair as two stores each covering whole lines of 8 samples (lanes s and s ^ 8 trade halves by a DPP
// row rotate: chain 3.73 -> 3.55 ms per mip step); the forward writes its pair as the two half-line
// stores back to back, no lane exchange (the exchange cost the forward ~0.2 ms; back to back:
// WRITE_SIZE 7.25 -> 6.47 GB per fine launch, step -0.08 ms, profiles/r03m).  Every chunk still
// issues 2 stores per column block (counted waits assume at least that many).

struct FusedArgs {
    nerf_fused_layer L[NERF_FUSED_MAX_LAYERS];
    nerf_fused_encoding enc[2];
    const char* img;
    int img_bytes;
    int gen_mask;      // bit e: encoding e is generated at the start of every tile (forward only)
    int gen_lds;       // the encoding the first layer reads from LDS (generated last), or -1
    int gen_reg;       // the encoding (one k-block) a later layer reads from the tile-start registers, or -1
    int n_layers;
    int M;
    int ntiles;
    int span;          // tiles a workgroup runs back to back (2: rays of 256 samples), ntiles % span == 0
    int comp_on;       // forward: composite every tile's rays (nerf_mlp_fused_render)
    nerf_fused_composite comp;
    // a generated hash-grid encoding (params.kind 2): its parameters, table and level row offsets
    nerf_hashgrid_params hg;
    const float* hg_table;
    int hg_off[16];
};
static_assert(sizeof(FusedArgs) <= 4096, "kernel arguments");

typedef __attribute__((address_space(4))) const char kchar_t;
typedef float* fptr_t;
typedef const float* cfptr_t;
typedef uint8_t* u8ptr_t;
typedef const uint8_t* cu8ptr_t;
// layer fields are read from the kernel-argument segment by scalar loads (indexing the by-value
// argument with a runtime layer index would make hipcc copy it to scratch)
#define LF(T, f, l)                                                                                          \
    (*(const __attribute__((address_space(4))) T*)(c.kargs + offsetof(FusedArgs, L) +                        \
                                                   (size_t)(l) * sizeof(nerf_fused_layer) +                  \
                                                   offsetof(nerf_fused_layer, f)))
#define LFI(T, f, i, l)                                                                                      \
    (*(const __attribute__((address_space(4))) T*)(c.kargs + offsetof(FusedArgs, L) +                        \
                                                   (size_t)(l) * sizeof(nerf_fused_layer) +                  \
                                                   offsetof(nerf_fused_layer, f) + (size_t)(i) * sizeof(T)))

// fields of encoding e (the generated HBM-fed segments), from the kernel-argument segment
#define EF(T, f, e)                                                                                          \
    (*(const __attribute__((address_space(4))) T*)(c.kargs + offsetof(FusedArgs, enc) +                      \
                                                   (size_t)(e) * sizeof(nerf_fused_encoding) +               \
                                                   offsetof(nerf_fused_encoding, f)))

// fields of the generated hash grid, from the kernel-argument segment
#define HG(T, f) (*(const __attribute__((address_space(4))) T*)(c.kargs + offsetof(FusedArgs, hg) +               \
                                                               offsetof(nerf_hashgrid_params, f)))

// fields of the fused composite, from the kernel-argument segment
#define CF(T, f)                                                                                             \
    (*(const __attribute__((address_space(4))) T*)(c.kargs + offsetof(FusedArgs, comp) +                    \
                                                   offsetof(nerf_fused_composite, f)))

__device__ __forceinline__ f4 mfma16(bf16x8 a, bf16x8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void split8(f8 v, bf16x8& hi, bf16x8& lo) {
    hi = __builtin_convertvector(v, bf16x8);
    lo = __builtin_convertvector(v - __builtin_convertvector(hi, f8), bf16x8);
}

__device__ __forceinline__ void barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ int n16_of(int N) { return (N + 15) >> 4; }

// Weight-fragment reads from the LDS ring by inline asm with explicitly counted waits.  hipcc
// cannot tell the ring slot being read from the one the LDS-DMA is filling, so for its own reads it
// waits for every outstanding DMA (vmcnt) and for every LDS read (lgkmcnt(0)), which empties the
// one-chunk-ahead prefetch.  The fragments pass through the wait statement, so no instruction can
// use them before it.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
template <int OFF>
__device__ __forceinline__ void lds_frag(bf16x8& f, unsigned addr) {
#ifndef NERF_FUSED_DIAG_NOFRAG     // diagnostic builds only: MFMAs on stale fragments, no LDS reads
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(addr), "n"(OFF));
#else
    asm volatile("; %1" : "=v"(f) : "v"(addr));
#endif
}
template <int N>
__device__ __forceinline__ void lds_wait(bf16x8& f0, bf16x8& f1) {
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(f0), "+v"(f1) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lds_wait1(bf16x8& f0) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(f0) : "n"(N));
}
// The HBM-fed weight fragments and the biases are inline-asm buffer loads waited for by explicit
// counts (hipcc's own wait for a buffer load in the chunk loop is vmcnt(0), which also waits for the
// DMA issued before it); the loaded values pass through the wait statements.
template <int N>
__device__ __forceinline__ void frag_vwait(bf16x8& f0, bf16x8& f1) {
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(f0), "+v"(f1) : "n"(N));
}
template <int N>
__device__ __forceinline__ void frag_vwait1(bf16x8& f0) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(f0) : "n"(N));
}
template <int N>
__device__ __forceinline__ void bias_wait(f4& b) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(b) : "n"(N));
}
__device__ __forceinline__ void buf_load16(f4& v, unsigned off, __amdgpu_buffer_rsrc_t r) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r));
}
__device__ __forceinline__ void buf_load16(bf16x8& v, unsigned off, __amdgpu_buffer_rsrc_t r) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r));
}

// t + t + !(x > 0): shifts the "dead ReLU" bit of x in (v_cmp + v_addc; plain C came out as
// compare, select and shift-or).  !(x > 0) holds for NaN, as the reference's (out > 0) is false.
__device__ __forceinline__ unsigned shift_in_dead(unsigned t, float x) {
    asm("v_cmp_nlt_f32 vcc, 0, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(t) : "v"(x) : "vcc");
    return t;
}

// kernel modes: the forward (bias, ReLU, mask bits and column outputs) and the backward's
// input-gradient chain (ReLU-bit multiply, second output for encoding rows; no bias)
constexpr int MODE_FWD = 0;
constexpr int MODE_DGRAD = 1;
constexpr int MODE_X1 = 2;

struct Ctx {
    kchar_t* kargs;
    char* smem;
    char* ximg;           // this wave's LDS image of the next layer's operand
    __amdgpu_buffer_rsrc_t rimg;
    int wave, lane, M, n_layers;
    int cur;              // ring slot of the next register-fed chunk
    // DMA cursor over the register-fed chunks of the network (layers with kbr = 0 have none); the
    // stream repeats per tile
    int d_off, d_units, d_left, d_layer;
    int d_remaining;      // chunks still to issue
    // per-layer DMA table, lane l = layer l (read by v_readlane: no scalar memory loads in the chunk
    // loop, whose out-of-order returns would force lgkmcnt(0) waits on the LDS reads)
    int t_off, t_units, t_n16, t_next;
    // the current layer's register-fed input (B operand): [32-deep k-block][16-sample column block]
    bf16x8 xh[KBMAX][SB], xl[KBMAX][SB];
    float dsink;          // diagnostic builds only
    // fused compositing (forward): the last layer's values (rows 4 g .. 4 g + 3), the density column
    // output and the interval length of the lane's samples (lanes g = 0)
    f4 head[SB];
    float sig[SB], cdist[SB];
    // rays of two tiles (S = 256): the first tile's heads and interval lengths, held over the second
    f4 phead[SB];
    float pcdist[SB];
    // the split k-block of encoding gen_reg for the wave's own samples, captured from the LDS rows at
    // the tile start and held across the layers (a later layer's generated segment, seg_gen on l > 0)
    bf16x8 gh[SB], gl[SB];
};

template <class CT>
__device__ __forceinline__ int dma_units(CT& c, int l) { return LF(int, chunk_units, l); }

// first layer at or after l (cyclically) with a register-fed part (kernel prologue only)
template <class CT>
__device__ __forceinline__ int next_ring_layer(CT& c, int l) {
    for (int i = 0; i < c.n_layers; ++i, l = (l + 1 == c.n_layers ? 0 : l + 1))
        if (dma_units(c, l) > 0) return l;
    return -1;
}

__device__ __forceinline__ void dma_seek(Ctx& c, int l) {
    c.d_layer = l;
    c.d_off = __builtin_amdgcn_readlane(c.t_off, l);
    c.d_units = __builtin_amdgcn_readlane(c.t_units, l);
    c.d_left = __builtin_amdgcn_readlane(c.t_n16, l);
}

// LDS-DMA (buffer_load_dwordx4 ... lds: image offset in an SGPR, the lane's 16 bytes in a constant
// VGPR) of the next register-fed chunk of the stream into ring slot `slot`: exactly DMA_PER_WAVE
// 1 KB pieces per wave, unconditionally (a chunk of 8 register-fed k-blocks is 16 pieces; smaller
// ones repeat pieces, and past the end of the stream the last chunk is fetched again), so that the
// count of vector-memory ops in a chunk is the same on every path
constexpr int DMA_PER_WAVE = 2 * KBMAX / NWAVE;
// (The same pieces by plain buffer loads into VGPRs and ds_write_b128 into the slot measured slower:
// step 12.53 vs 12.22 ms, profiles/r04e.)
__device__ __forceinline__ void dma_advance(Ctx& c) {
    if (c.d_remaining > 1) {
        c.d_off += c.d_units * 1024;
        if (--c.d_left == 0) dma_seek(c, __builtin_amdgcn_readlane(c.t_next, c.d_layer));
        --c.d_remaining;
    }
}
__device__ __forceinline__ void issue_dma(Ctx& c, int slot) {
    char* dst = c.smem + slot * SLOT_BYTES;
#ifndef NERF_FUSED_DIAG_NODMA          // diagnostic builds only: time the kernel without its weight stream
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; ++i) {
        const int u = (c.wave + NWAVE * i) & (c.d_units - 1);   // d_units: 8 or 16
        __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rimg, (lds_void_t*)(dst + u * 1024), 16, c.lane * 16,
                                                 c.d_off + u * 1024, 0, 0);
    }
#else
    (void)dst;
#endif
    dma_advance(c);
}

// Arguments of the shared encoding math (encode_common.h) for a generated segment: the encoding's
// parameters stay in the kernel-argument segment (uniform fields are scalar loads; the per-level
// mask is indexed per lane and read from there too, never copied to private memory)
struct GenArgs {
    const __attribute__((address_space(4))) nerf_pe_params& p;
    const float *x, *xdir, *o, *d, *t0, *t1, *pw;
    int S;
    int64_t n_rays;
};

// Rows of encoding e for the wave's NS samples base .. base + NS - 1, written into LDS (the wave's
// operand-image region, unused before a layer's chunk loop): row r, columns [0, 64) (zeros past
// out_dim), as nerf_encode_fwd computes them (the same encode_common.h functions, fp contraction
// off: bitwise equal).  The wave shares the work like encode_fwd_lds_kernel: per-sample terms
// (position, IPE mean shift and variances) once per sample, then one sincos per (sample, d, k)
// task for both its cos and sin columns.  Rows past M hold values of a zero position (their
// outputs are dropped).
constexpr int GEN_LD = 68;                    // floats per LDS row: 64 columns + 16-B pad
static_assert(SPW * (GEN_LD + 8) * 4 <= XIMG_BYTES, "generator scratch");
// The per-sample inputs of encoding e for lanes < NS (sample base + lane): o xyz, d xyz, t0, t1,
// pixel width for ray-mode positions; x xyz for per-ray directions.  Loads only, so that the
// tile's inputs of both encodings are in flight together (one memory round trip per tile).
template <int NS, class CT>
__device__ __forceinline__ void gen_load(const CT& c, int e, int base, float (&v)[9]) {
#pragma unroll
    for (int j = 0; j < 9; ++j) v[j] = 0.f;
    const int m = base + c.lane;
    if (c.lane >= NS || m >= c.M) return;
    const int per_ray = EF(int, per_ray, e);
    const unsigned S = (unsigned)EF(int, samples_per_ray, e);
    const float* ray_d = EF(cfptr_t, ray_d, e);
    const int64_t ray = (int64_t)((unsigned)m / S);
    if (per_ray) {
        v[0] = ray_d[ray * 3 + 0]; v[1] = ray_d[ray * 3 + 1]; v[2] = ray_d[ray * 3 + 2];
        return;
    }
    const float* o = EF(cfptr_t, ray_o, e);
    const __attribute__((address_space(4))) nerf_pe_params& p = EF(nerf_pe_params, params, e);
    v[0] = o[ray * 3 + 0]; v[1] = o[ray * 3 + 1]; v[2] = o[ray * 3 + 2];
    v[3] = ray_d[ray * 3 + 0]; v[4] = ray_d[ray * 3 + 1]; v[5] = ray_d[ray * 3 + 2];
    v[6] = EF(cfptr_t, t_start, e)[m];
    if (p.query != 0 || p.kind == 1) v[7] = EF(cfptr_t, t_end, e)[m];
    const float* pw = EF(cfptr_t, pixel_width, e);
    if (p.kind == 1 && pw != nullptr) {
        const GenArgs a{p, nullptr, nullptr, o, ray_d, nullptr, nullptr, pw, (int)S, EF(int64_t, n_rays, e)};
        v[8] = pixel_width_at(a, m);
    }
}

// Hash-grid features (params.kind 2) of the wave's samples into its LDS scratch, as
// hashgrid_fwd_tile_kernel computes them (hashgrid_common.h: the same corner arithmetic, the 8
// corners' feature loads issued before the sums, products rounded then added in corner order):
// the samples' positions first (lanes < NS), then one level per trip.
template <int NS, class CT>
__device__ __forceinline__ void gen_hash_rows(const CT& c, int base, const float (&v)[9]) {
#pragma clang fp contract(off)
    float* R = reinterpret_cast<float*>(c.ximg);          // [NS][GEN_LD]
    float* P = R + NS * GEN_LD;                             // [NS][8]: position xyz
    const int L = HG(int32_t, levels), F = HG(int32_t, features), T = HG(int32_t, table_size);
    const int cols = L * F;
    if (c.lane < NS) {
        float p[3] = {0.f, 0.f, 0.f};
        if (base + c.lane < c.M) {
            // as sample_position (hashgrid.hip): o + tq d
            const float tq = HG(int32_t, query) == 0 ? v[6] : (v[6] + v[7]) / 2.0f;
            p[0] = v[0] + tq * v[3];
            p[1] = v[1] + tq * v[4];
            p[2] = v[2] + tq * v[5];
        }
        float* pr = P + c.lane * 8;
        pr[0] = p[0]; pr[1] = p[1]; pr[2] = p[2];
        float* row = R + c.lane * GEN_LD;
        for (int col = cols; col < 64; ++col) row[col] = 0.f;
    }
    // (same wave: its LDS operations complete in order, so the positions above are visible below)
    // One level per trip, its resolution and row offset uniform (scalar loads), lane s < NS on
    // sample s: bitwise the stand-alone kernel and repeatable on both corner forms
    // (tests/test_hashgrid.py).  Round 4 also ran four levels per trip (16-lane groups, per-lane
    // level parameters); with the int64 corner arithmetic of that time it dropped corner 2's term
    // at random in the last trip's fourth group of waves 4-7 — localised by bisection to that
    // compiled form, not reproduced with the current corner code.
    const int normalize = HG(int32_t, normalize);
    const __attribute__((address_space(4))) int64_t* primes =
        (const __attribute__((address_space(4))) int64_t*)(c.kargs + offsetof(FusedArgs, hg) +
                                                           offsetof(nerf_hashgrid_params, primes));
    const long long pr[3] = {(long long)primes[0], (long long)primes[1], (long long)primes[2]};
    const __attribute__((address_space(4))) int32_t* res =
        (const __attribute__((address_space(4))) int32_t*)(c.kargs + offsetof(FusedArgs, hg) +
                                                           offsetof(nerf_hashgrid_params, res));
    const __attribute__((address_space(4))) int* offs =
        (const __attribute__((address_space(4))) int*)(c.kargs + offsetof(FusedArgs, hg_off));
    const float* table = *(const __attribute__((address_space(4))) cfptr_t*)(c.kargs + offsetof(FusedArgs, hg_table));
    for (int l = 0; l < L; ++l) {
        const int rl = res[l], ol = offs[l];
        if (c.lane < NS) {
            const int r = c.lane;
            const float p[3] = {P[r * 8 + 0], P[r * 8 + 1], P[r * 8 + 2]};
            const Corners cn = level_corners(p, normalize, rl, T, pr);
            const float* tab = table + (int64_t)ol * F;
            float* o = R + r * GEN_LD + l * F;
            float g[8][4];
#pragma unroll
            for (int k = 0; k < 8; ++k)          // the 8 corners' feature loads before the sums
#pragma unroll
                for (int f = 0; f < 4; ++f) g[k][f] = f < F ? tab[(int64_t)cn.idx[k] * F + f] : 0.f;
            float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int f = 0; f < 4; ++f) acc[f] = acc[f] + cn.w[k] * g[k][f];
#pragma unroll
            for (int f = 0; f < 4; ++f)
                if (f < F) o[f] = acc[f];
        }
    }
}

// Rows of encoding e from its inputs (gen_load) into the wave's LDS scratch.
template <int NS, class CT>
__device__ __forceinline__ void gen_rows_lds(const CT& c, int e, int base, const float (&v)[9]) {
#pragma clang fp contract(off)
    float* R = reinterpret_cast<float*>(c.ximg);          // [NS][GEN_LD]
    float* P = R + NS * GEN_LD;                             // [NS][8]: pm xyz, vb xyz
    const __attribute__((address_space(4))) nerf_pe_params& prm = EF(nerf_pe_params, params, e);
    if (prm.kind == 2) {
        gen_hash_rows<NS>(c, base, v);
        return;
    }
    const int per_ray = EF(int, per_ray, e);
    const int out_dim = EF(int, out_dim, e);
    const int L = prm.levels, id = prm.include_identity ? 3 : 0;
    if (c.lane < NS) {
        float pm[3] = {0.f, 0.f, 0.f}, vb[3] = {0.f, 0.f, 0.f};
        if (base + c.lane < c.M) {
            // as load_pos_dir (encode_common.h): x, or o + tq d
            float p[3], dv[3];
            if (per_ray) {
                p[0] = v[0]; p[1] = v[1]; p[2] = v[2];
                dv[0] = dv[1] = dv[2] = 0.f;
            } else {
                const float tq = prm.query == 0 ? v[6] : (v[6] + v[7]) / 2.0f;
                dv[0] = v[3]; dv[1] = v[4]; dv[2] = v[5];
                p[0] = v[0] + tq * dv[0];
                p[1] = v[1] + tq * dv[1];
                p[2] = v[2] + tq * dv[2];
            }
            if (prm.kind == 1) {
                const IpeSample q = ipe_sample(prm, p, dv, v[6], v[7], v[8]);
                pm[0] = q.pm[0]; pm[1] = q.pm[1]; pm[2] = q.pm[2];
                vb[0] = q.vb[0]; vb[1] = q.vb[1]; vb[2] = q.vb[2];
            } else {
                pm[0] = p[0]; pm[1] = p[1]; pm[2] = p[2];
            }
        }
        float* pr = P + c.lane * 8;
        pr[0] = pm[0]; pr[1] = pm[1]; pr[2] = pm[2];
        pr[3] = vb[0]; pr[4] = vb[1]; pr[5] = vb[2];
        float* row = R + c.lane * GEN_LD;
        for (int col = 0; col < id; ++col) row[col] = pm[col];
        for (int col = out_dim; col < 64; ++col) row[col] = 0.f;
    }
    // (same wave: its LDS operations complete in order, so the terms above are visible below)
    const int na = 3 * L;
    // lane (r, g) = (lane % NS, lane / NS) takes sample r's tasks j = g, g + 64 / NS, ...: the
    // sample's terms read once, no division, the mask value of level k from lane k (ds_bpermute;
    // lanes 0-15 have g = 0 and so take part in every trip)
    {
        // the mask value of level k is read from lane k: lanes 0-15 hold levels 0-15 (encoding_ok caps
        // levels at 16, the 64-column LDS row at 10) and must all be in group g = 0
        static_assert(NS >= 16 && NS <= 64 && 64 % NS == 0, "mask lanes 0-15 in the g = 0 group");
        constexpr int G = 64 / NS;
        const int r = c.lane % NS, g = c.lane / NS;
        const float* pr = P + r * 8;
        const float pmr[3] = {pr[0], pr[1], pr[2]}, vbr[3] = {pr[3], pr[4], pr[5]};
        const float mreg = prm.use_mask ? prm.mask[c.lane & 15] : 1.f;
        const float scale = prm.scale;
        const int kind = prm.kind, use_mask = prm.use_mask;
        float* row = R + r * GEN_LD + id;
        for (int j = g; j < na; j += G) {
            const int dd = j >= 2 * L ? 2 : (j >= L ? 1 : 0);
            const int k = j - dd * L;
            const float sc = scale * (float)(1u << k);
            float sn, cs;
            sincos_enc(sel3(pmr, dd) * sc, &sn, &cs);
            if (kind == 1) {
                // mip-NeRF weight exp(-(var_d * 4^k) / 2) (positional_encodings.py:213-232)
                const float w = expf((-(sel3(vbr, dd) * (float)(1u << (2 * k)))) / 2.0f);
                cs = cs * w;
                sn = sn * w;
            }
            if (use_mask) {
                const float mk = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(k << 2, __builtin_bit_cast(int, mreg)));
                cs = mk * cs;
                sn = mk * sn;
            }
            row[j] = cs;
            row[na + j] = sn;
        }
    }
}

// The generated rows of the wave's samples into the encoding's rows in HBM (read back by later
// layers of the launch and by the weight gradients; a per-ray encoding by the ray's first sample):
// each instruction stores 1 KB of consecutive 16-byte row pieces.
template <int NS, class CT>
__device__ __forceinline__ void gen_store(const CT& c, int e, int base) {
    const float* R = reinterpret_cast<const float*>(c.ximg);
    float* out = EF(fptr_t, out, e);
    const int per_ray = EF(int, per_ray, e);
    const unsigned S = (unsigned)EF(int, samples_per_ray, e);
    const int ld = (int)EF(int64_t, ld, e);
    const int q4 = ld >> 2;                                   // 16-byte pieces per row (ld <= 64)
    for (int i = c.lane; i < NS * q4; i += 64) {
        const int r = i / q4, q = i - r * q4;
        const int m = base + r;
        if (m < c.M && (!per_ray || (unsigned)m % S == 0u)) {
            const int64_t n = per_ray ? (int64_t)((unsigned)m / S) : (int64_t)m;
            *reinterpret_cast<f4*>(out + n * ld + 4 * q) = *reinterpret_cast<const f4*>(R + r * GEN_LD + 4 * q);
        }
    }
}

// Columns col .. col + 7 of generated row r (gen_rows_lds), split into the bf16 hi/lo operand halves.
template <class CT>
__device__ __forceinline__ void gen_block(const CT& c, int r, int col, bf16x8& h, bf16x8& lo) {
    const float* R = reinterpret_cast<const float*>(c.ximg) + r * GEN_LD + col;
    const f4 v0 = *reinterpret_cast<const f4*>(R), v1 = *reinterpret_cast<const f4*>(R + 4);
    split8(__builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7), h, lo);
}

// Input rows of a chain step fed by the fused composite (seg_gen 3: head gradient, 4: density
// gradient; include/nerf_amd.h nerf_fused_composite): per sample the coefficient row (coef [M][8])
// times its ray's grad_rgb, stored for the weight gradients and split into the B operand of the
// step's k-block (lanes g = 0 hold columns 0..7, the others zeros).
__device__ __forceinline__ void comp_grad_block(const Ctx& c, int gen, const float* coef, const int (&sample)[SB],
                                                const bool (&row_ok)[SB], bf16x8 (&h)[SB], bf16x8 (&lo)[SB]) {
#pragma clang fp contract(off)
    const unsigned S = (unsigned)CF(int32_t, samples_per_ray);
    const float* grgb = CF(cfptr_t, grad_rgb);
    const bool dens_head = CF(int32_t, sigma_layer) < 0;
    float* out = gen == 3 ? CF(fptr_t, grad_head) : CF(fptr_t, grad_sigma);
    const int64_t ldo = gen == 3 ? CF(int64_t, ld_head) : CF(int64_t, ld_sigma);
#pragma unroll
    for (int sb = 0; sb < SB; ++sb) {
        f4 x0 = {0.f, 0.f, 0.f, 0.f};
        if ((c.lane >> 4) == 0 && row_ok[sb]) {
            const unsigned m = (unsigned)sample[sb];
            const unsigned ray = m / S;
            const f4 q0 = *reinterpret_cast<const f4*>(coef + (size_t)m * 8);
            const f4 q1 = *reinterpret_cast<const f4*>(coef + (size_t)m * 8 + 4);
            const float g0 = grgb[ray * 3 + 0], g1 = grgb[ray * 3 + 1], g2 = grgb[ray * 3 + 2];
            const float ds = (g0 * q1[0] + g1 * q1[1]) + g2 * q1[2];
            if (gen == 3)
                x0 = f4{g0 * q0[0], g1 * q0[1], g2 * q0[2], dens_head ? ds : 0.f};
            else
                x0 = f4{ds, 0.f, 0.f, 0.f};
            // nontemporal, as the layer outputs: the first chunk's vmcnt(0) waits for its acknowledgement
            if (out != nullptr) __builtin_nontemporal_store(x0, reinterpret_cast<f4*>(out + (size_t)m * ldo));
        }
        split8(__builtin_shufflevector(x0, f4{0.f, 0.f, 0.f, 0.f}, 0, 1, 2, 3, 4, 5, 6, 7), h[sb], lo[sb]);
    }
}

struct LayerState {
    int floor_i;          // ReLU as an integer max on the fp32 bits: 0, or INT_MIN for no ReLU
    int col_chunk;        // 16-row chunk holding the column output (-1: none)
    int n1;               // 16-row chunks routed to out (fed forward, masked); the rest go to out2
    unsigned bias_off;
    unsigned row_off[SB];     // byte offset of this lane's 4 columns of chunk 0 in out (OOB past M)
    unsigned row_off2[SB];    // ... in out2 (chunk n1)
    int colok, colok2;        // ldo - 4 g: chunk ch is in range while 16 ch < colok
    unsigned sample_off[SB];  // sample * 4 for lane group 0 (OOB otherwise / past M)
    unsigned mrow_off[SB];    // this lane's 8 bytes of the sample's mask row (OOB past M)
    __amdgpu_buffer_rsrc_t ro, rm, rc, ro2;
    unsigned mw[SB][2];   // this lane's ReLU mask words (NERF_FUSED_MASK layout; [1] accumulates)
    f4 stash[SB];             // the even chunk's values, stored with the odd chunk's
    unsigned pa[SB], pb[SB];  // row offsets (+16 g) of the samples this lane writes in the pair's
    unsigned pa2[SB], pb2[SB];  // stores A (samples 0-7 of the block) and B (8-15), in out / out2
    int last_even;            // NC - 1 for an odd chunk count (stored alone), else -1
    unsigned mi[SB][2];   // mask_in: this lane's two words of the sample's bits (NERF_FUSED_MASK layout)
    unsigned mcur[SB];    // the word of the current chunk (mi[0], mi[1] from chunk 8, zero past n1)
};

// hi = bf16(v), lo = bf16(v - hi) of two values, packed (the rounded pair's halves read back as fp32
// by a shift / a mask instead of a second conversion)
__device__ __forceinline__ void split2(float x, float y, unsigned& hi, unsigned& lo) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    const bf16x2 h = __builtin_convertvector((f4{x, y, 0.f, 0.f}).xy, bf16x2);
    hi = __builtin_bit_cast(unsigned, h);
    // one packed subtract (exact: hi is x rounded).  Scalar subtracts / no SLP packing anywhere in
    // the kernel (no v_pk_*_f32 beside the MFMAs) measured within noise: step 11.33 / 11.24 vs
    // 11.26 ms, three rotating repetitions (profiles/r06f)
    const f2 hf = {__builtin_bit_cast(float, hi << 16), __builtin_bit_cast(float, hi & 0xffff0000u)};
    const f2 d = f2{x, y} - hf;
    lo = __builtin_bit_cast(unsigned, __builtin_convertvector(d, bf16x2));
}

// bf16(x), bf16(y) packed (round to nearest even: the hi half of split2)
__device__ __forceinline__ unsigned hi2(float x, float y) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f4{x, y, 0.f, 0.f}).xy, bf16x2));
}

__device__ __forceinline__ bool pair_odd(int ch) { return ch >= 0 && (ch & 1) != 0; }

__device__ __forceinline__ float ror8(float x) {      // lane (s ^ 8) of this lane's 16-lane row
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x128, 0xf, 0xf, false));
}

// The two stores of chunk pair (ch - 1, ch), ch odd (chunk indices local to the output): lane (s, g)
// holds x = columns 4 g .. 4 g + 3 of chunk ch - 1 (stashed) and y = those of chunk ch, for sample
// s.  Store A writes the whole 128-B line segment of samples 0-7 (lanes s < 8: their own x; lanes
// s >= 8: y of sample s - 8), store B that of samples 8-15 (lanes s < 8: x of sample s + 8; lanes
// s >= 8: their own y).
__device__ __forceinline__ void pair_stores(const Ctx& c, const LayerState& st, int sb, int ch, int colok,
                                            unsigned pa, unsigned pb, const f4& y, f4& va, f4& vb, unsigned& oa,
                                            unsigned& ob) {
    const f4 x = st.stash[sb];
    const bool lo8 = (c.lane & 8) == 0;
    f4 rx, ry;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float xr = x[r], yr = y[r];
        rx[r] = ror8(xr);
        ry[r] = ror8(yr);
    }
    va = lo8 ? x : ry;
    vb = lo8 ? rx : y;
    const int cl = lo8 ? ch - 1 : ch;                 // the chunk this lane writes in both stores
    const bool inr = cl >= 0 && 16 * cl < colok;
    oa = inr ? pa + 64u * (unsigned)cl : OOB;
    ob = inr ? pb + 64u * (unsigned)cl : OOB;
}

// Epilogue of 16-row chunk ch (output rows 16 ch .. 16 ch + 15; ch = -1: none, the stores are
// dropped), in four parts placed between the next chunk's MFMA stages: 0 / 1 = the values of column
// block 0 / 1 (FWD: bias + ReLU; DGRAD: times the ReLU bits) and their fp32 stores; 2 = ReLU mask
// bits (FWD); 3 = the hi/lo split into the LDS image of the next layer's operand.
// EPAR: the parity of chunk ch when the caller knows it at compile time (the chunk loop unrolled by
// two: 0 even, 1 odd — ch = -1, the nonexistent predecessor of chunk 0, comes in the odd slot with
// every store dropped), -1: decided at run time
template <int MODE, int EPAR = -1>
__device__ __forceinline__ void epi_part(Ctx& c, LayerState& st, int p, int ch, f4 (&a)[SB], f4 b) {
#ifdef NERF_FUSED_DIAG_NOEPI           // diagnostic builds only (timing without the chunk epilogues)
    return;
#endif
#ifdef NERF_FUSED_DIAG_MFMAONLY   // diagnostic: the epilogue reduced to one add (the MFMAs stay live)
    if (p == 0) c.dsink += a[0][0] + a[0][3];
    return;
#endif
#ifdef NERF_FUSED_DIAG_NOMASK     // diagnostic: no ReLU mask bits
    if (p == 2) return;
#endif
#ifdef NERF_FUSED_DIAG_NOSPLIT    // diagnostic: no next-operand split / image writes
    if (p == 3) return;
#endif
    const int q = ch >> 1, bb = ch & 1;
    if (p < 2) {
        if (p >= SB) return;
        const int sb = p;
        f4& v = a[sb];
        if constexpr (is_fwd(MODE)) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                v[r] = __builtin_bit_cast(float, max(__builtin_bit_cast(int, v[r] + b[r]), st.floor_i));
            if (ch >= 0 && ch == st.col_chunk) c.sig[sb] = v[0];   // (the raw density, for fused compositing)
            if (EPAR >= 0 ? EPAR == 0 : !pair_odd(ch)) {
                // even chunk: held for the pair (alone if it is the layer's last); the column output
                // (col_idx is a multiple of 32: always an even chunk)
                st.stash[sb] = v;
                const unsigned off =
                    ch >= 0 && ch == st.last_even && 16 * ch < st.colok ? st.row_off[sb] + 64u * (unsigned)ch : OOB;
                __builtin_amdgcn_raw_buffer_store_b128(v, st.ro, off, 0, ST_AUX);
                const unsigned coff = ch == st.col_chunk ? st.sample_off[sb] : OOB;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[0]), st.rc, coff, 0, 0);
            } else {
                // the pair's two half lines of every sample back to back (the even chunk's from the stash):
                // no lane exchange, the halves reach L2 together
                const unsigned oa = ch > 0 && 16 * (ch - 1) < st.colok ? st.row_off[sb] + 64u * (unsigned)(ch - 1) : OOB;
                const unsigned ob = ch >= 0 && 16 * ch < st.colok ? st.row_off[sb] + 64u * (unsigned)ch : OOB;
                __builtin_amdgcn_raw_buffer_store_b128(st.stash[sb], st.ro, oa, 0, ST_AUX);
                __builtin_amdgcn_raw_buffer_store_b128(v, st.ro, ob, 0, ST_AUX);
            }
        } else {
            const bool sec = ch >= st.n1;          // an encoding input's rows (out2): not masked
            // column 16 ch + 4 g + r is (dead) bit 4 (7 - (ch & 7)) + r of this lane's word ch >> 3 (zero
            // without mask_in: an empty buffer reads 0); chunks come in order, so the layer switches
            // mcur twice by uniform branches (to word 1 at chunk 8, to zero at the first out2 chunk).
            // No chunk before 0 (its stores are dropped): the words are first read in the second
            // chunk, after its DMA wait has covered their load
            const int sh = 4 * (7 - (ch & 7));
            if (ch == 8 && ch < st.n1) st.mcur[sb] = st.mi[sb][1];
            if (ch == st.n1) st.mcur[sb] = 0u;
#ifndef NERF_FUSED_DIAG_NOMASKIN   // diagnostic: the ReLU bits not applied
            if (ch >= 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int dead = __builtin_amdgcn_sbfe((int)st.mcur[sb], (unsigned)(sh + r), 1u);   // 0 / -1
                    // (through a scalar: __builtin_bit_cast of the vector element lvalue v[r] reads element 0)
                    const float x = v[r];
                    v[r] = __builtin_bit_cast(float, __builtin_bit_cast(int, x) & ~dead);
                }
            }
#else
            (void)sh;
#endif
#ifdef NERF_FUSED_DIAG_NOSTORE
            return;
#endif
#ifdef NERF_FUSED_DIAG_DROPSTORE       // diagnostic: every chain store addressed past the buffer
            st.colok = st.colok2 = -1 << 20;
            st.pa[sb] = st.pb[sb] = st.pa2[sb] = st.pb2[sb] = st.row_off[sb] = st.row_off2[sb] = OOB;
#endif
            if (EPAR >= 0 ? EPAR == 0 : !pair_odd(ch)) {
                // even chunk: held for the pair (alone if it is the layer's last); n1 is even, so
                // both chunks of a pair go to the same output
                st.stash[sb] = v;
                const bool alone = ch >= 0 && ch == st.last_even;
                const unsigned off1 = alone && !sec && 16 * ch < st.colok ? st.row_off[sb] + 64u * (unsigned)ch : OOB;
                const unsigned off2 =
                    alone && sec && 16 * (ch - st.n1) < st.colok2 ? st.row_off2[sb] + 64u * (unsigned)(ch - st.n1) : OOB;
                __builtin_amdgcn_raw_buffer_store_b128(v, st.ro, off1, 0, ST_AUX);
                __builtin_amdgcn_raw_buffer_store_b128(v, st.ro2, off2, 0, ST_AUX);
            } else if (!sec) {
                f4 va, vb;
                unsigned oa, ob;
                pair_stores(c, st, sb, ch, st.colok, st.pa[sb], st.pb[sb], v, va, vb, oa, ob);
                __builtin_amdgcn_raw_buffer_store_b128(va, st.ro, oa, 0, ST_AUX);
                __builtin_amdgcn_raw_buffer_store_b128(vb, st.ro, ob, 0, ST_AUX);
            } else {
                f4 va, vb;
                unsigned oa, ob;
                pair_stores(c, st, sb, ch - st.n1, st.colok2, st.pa2[sb], st.pb2[sb], v, va, vb, oa, ob);
                __builtin_amdgcn_raw_buffer_store_b128(va, st.ro2, oa, 0, ST_AUX);
                __builtin_amdgcn_raw_buffer_store_b128(vb, st.ro2, ob, 0, ST_AUX);
            }
        }
    } else if (p == 2) {
        if constexpr (is_fwd(MODE)) {
            // NERF_FUSED_MASK layout: the lane's own bits, no cross-lane step.  The bits of rows
            // 4 g + r of chunks 0-7 / 8-15 shift into a word of their own, !(a > 0) entering as the
            // carry of t + t (two VALU per value; the NERF_EPI_MASKOUT layout's per-sample words
            // took an OR across the lane groups and a word select: ~20 VALU per chunk, and the
            // chain 8 words per sample).  Bits mark dead units, so that an absent mask reads as 0.
            if (ch >= 0 && ch < 2 * KBMAX) {
#pragma unroll
                for (int sb = 0; sb < SB; ++sb) {
                    unsigned t = st.mw[sb][1];
#pragma unroll
                    for (int r = 3; r >= 0; --r) t = shift_in_dead(t, a[sb][r]);
                    st.mw[sb][1] = t;
                }
                if (ch == 7) {
#pragma unroll
                    for (int sb = 0; sb < SB; ++sb) {
                        st.mw[sb][0] = st.mw[sb][1];
                        st.mw[sb][1] = 0;
                    }
                }
            }
        }
    } else {
        // rows 16 bb + 4 g + r of k-block q of the next layer = elements 4 bb + r of lane (s, g):
        // 8 bytes of the lane's 16-byte hi and lo slots (chunks past the fed outputs are not written)
        if (ch >= 0 && ch < 2 * KBMAX && ch < st.n1) {
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) {
                typedef unsigned u2 __attribute__((ext_vector_type(2)));
                char* d = c.ximg + ((q * SB + sb) * 2) * 1024 + c.lane * 16 + 8 * bb;
                if constexpr (is_x1(MODE)) {
                    // the next layer's operand rounded once (the lo half is never read)
                    *reinterpret_cast<u2*>(d) = u2{hi2(a[sb][0], a[sb][1]), hi2(a[sb][2], a[sb][3])};
                } else {
                    unsigned h0, l0, h1, l1;
                    split2(a[sb][0], a[sb][1], h0, l0);
                    split2(a[sb][2], a[sb][3], h1, l1);
                    const u2 h = {h0, h1}, lo = {l0, l1};
                    *reinterpret_cast<u2*>(d) = h;
                    *reinterpret_cast<u2*>(d + 1024) = lo;
                }
            }
        }
    }
}

// Epilogue parts in the MFMA stream: the parts that do anything (1 only with SB = 2) go to
// consecutive register-fed stages from EPI0 on, part 3 (the hi/lo split into the next layer's
// operand image) included; parts that do not fit run after the chunk's HBM-fed MFMAs
constexpr int EPI_NP = 3;                                      // parts placed in stages
__host__ __device__ constexpr int epi_part_of(int i) {         // i-th placed part (part 1: SB = 2 only)
    return i == 0 ? 0 : i + 1;
}
template <int KBR, int EPI0>
__host__ __device__ constexpr int epi_placed() {                 // parts placed in the stages
    return KBR - EPI0 < EPI_NP ? (KBR - EPI0 > 0 ? KBR - EPI0 : 0) : EPI_NP;
}

// the first k-step of an 8-block chunk carrying the previous chunk's epilogue (its bias waited
// there): forward 3, chain 4.  One box, three rotating repetitions (profiles/r05x), ms per step
// forward / chain: 1: 3.84 / 3.44, 2: 3.83 / 3.42, 3: 3.77 / 3.41, 4: 3.89 / 3.39
template <int MODE>
constexpr int epi0_of() { return is_fwd(MODE) ? 3 : 4; }

// k-steps of weight fragments read ahead of the step being multiplied
// (3 or 4 steps ahead for the single pass, whose hi-only fragments leave the registers for it:
// n2v forward 0.968 / 0.967 ms per step vs 0.968 at 2, three rotating repetitions, profiles/r06g)
constexpr int FA = 2;

// the chunk's first min(FA, KBR) steps' fragment reads (compile-time LDS offsets; the hi halves
// only in a single-pass mode)
template <int MODE, int KBR, int I>
__device__ __forceinline__ void first_reads(bf16x8 (&fr)[FA][2], unsigned sa) {
    if constexpr (I < FA && I < KBR) {
        lds_frag<I * 2048>(fr[I][0], sa);
        if constexpr (!is_x1(MODE)) lds_frag<I * 2048 + 1024>(fr[I][1], sa);
        first_reads<MODE, KBR, I + 1>(fr, sa);
    }
}

// One 16-row chunk's register-fed k-blocks (compile-time KB_I: immediate LDS offsets), fragments
// read FA steps ahead; the previous chunk's epilogue parts 0-2 at stages EPI0 .. EPI0 + 2.
template <int MODE, int KBR, int KBH, int KB_I, int EPAR = -1>
__device__ __forceinline__ void reg_steps(Ctx& c, LayerState& st, unsigned sa, bf16x8 (&fr)[FA][2], f4 (&a)[SB],
                                          f4 (&pv)[SB], f4& pb, int ch) {
    constexpr int EPI0 = KBR >= 8 ? epi0_of<MODE>() : (KBR >= 4 ? 1 : 0);
    if constexpr (KB_I < KBR) {
        bf16x8(&f)[2] = fr[KB_I % FA];
        // this step's fragments have landed (the reads of the steps after it may still be in flight)
        constexpr int later = (KB_I + FA - 1 < KBR - 1 ? KB_I + FA - 1 : KBR - 1) - KB_I;
        // (epilogue part 3's operand-image writes in the previous stage may land on either side of
        // that stage's fragment reads — the asm reads carry no memory clobber — so they are not
        // counted as younger: waiting for them too is the safe side)
        if constexpr (is_x1(MODE)) {
            lds_wait1<later>(f[0]);
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(f[0], c.xh[KB_I][sb], a[sb]);
        } else {
            lds_wait<2 * later>(f[0], f[1]);
            // products lo*hi + hi*lo + hi*hi per accumulator (small terms first, as linear_x3.hip)
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(f[1], c.xh[KB_I][sb], a[sb]);
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(f[0], c.xl[KB_I][sb], a[sb]);
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(f[0], c.xh[KB_I][sb], a[sb]);
        }
        if constexpr (KB_I + FA < KBR) {
            lds_frag<(KB_I + FA) * 2048>(f[0], sa);
            if constexpr (!is_x1(MODE)) lds_frag<(KB_I + FA) * 2048 + 1024>(f[1], sa);
        }
        // (placing the epilogue parts of the two waves of a SIMD at different stages, 0-2 and 4-6,
        // measured slower: chain 3.78 -> 4.03-4.09 ms, forward 3.86 -> 3.94-4.00 per mip step)
        if constexpr (KB_I == EPI0 && is_fwd(MODE))
            bias_wait<(KBR > 0 ? DMA_PER_WAVE : 0) + (is_x1(MODE) ? 1 : 2) * KBH>(pb);   // (younger: the DMA, the HBM fragments)
        if constexpr (KB_I >= EPI0 && KB_I < EPI0 + epi_placed<KBR, EPI0>())
            epi_part<MODE, EPAR>(c, st, epi_part_of(KB_I - EPI0), ch - 1, pv, pb);
        __builtin_amdgcn_sched_barrier(0);
        reg_steps<MODE, KBR, KBH, KB_I + 1, EPAR>(c, st, sa, fr, a, pv, pb, ch);
    }
}

// One layer of shape (KBR register-fed, KBH HBM-fed 32-deep k-blocks): runtime loop over its
// 16-row output chunks.
template <int MODE, int KBR, int KBH>
__device__ __forceinline__ void fused_layer(Ctx& c, int l, int base) {
    constexpr int EPI0 = KBR >= 8 ? epi0_of<MODE>() : (KBR >= 4 ? 1 : 0);   // first stage carrying an epilogue part
    const int g = c.lane >> 4;
    const int N = LF(int, N, l);
    const int NC = n16_of(N);
    LayerState st;
    const int ldo = (int)LF(int64_t, ldo, l);
    st.floor_i = LF(int, relu, l) != 0 ? 0 : (int)0x80000000;
    st.colok = ldo - 4 * g;
    st.last_even = (NC & 1) ? NC - 1 : -1;
    int sample[SB];
    bool row_ok[SB];
#pragma unroll
    for (int sb = 0; sb < SB; ++sb) {
        sample[sb] = base + 16 * sb + (c.lane & 15);
        row_ok[sb] = sample[sb] < c.M;
        st.row_off[sb] = row_ok[sb] ? (unsigned)sample[sb] * (unsigned)ldo * 4u + 16u * g : OOB;
        st.sample_off[sb] = row_ok[sb] && g == 0 ? (unsigned)sample[sb] * 4u : OOB;
        st.mrow_off[sb] = row_ok[sb] ? (unsigned)sample[sb] * 32u + 8u * g : OOB;
        {
            const int sa = (c.lane & 8) == 0 ? sample[sb] : sample[sb] - 8;   // store A's sample
            const int sbb = sa + 8;                                           // store B's
            st.pa[sb] = sa < c.M ? (unsigned)sa * (unsigned)ldo * 4u + 16u * g : OOB;
            st.pb[sb] = sbb < c.M ? (unsigned)sbb * (unsigned)ldo * 4u + 16u * g : OOB;
        }
        st.mw[sb][0] = st.mw[sb][1] = 0;
    }
    st.ro = __builtin_amdgcn_make_buffer_rsrc(LF(fptr_t, out, l), 0, c.M * ldo * 4, RSRC_W3);
    st.bias_off = (unsigned)LF(int64_t, bias_off, l) + 16u * g;
    if constexpr (is_fwd(MODE)) {
        uint8_t* mptr = LF(u8ptr_t, mask, l);
        st.rm = __builtin_amdgcn_make_buffer_rsrc(mptr, 0, mptr != nullptr ? c.M * 32 : 0, RSRC_W3);
        float* cptr = LF(fptr_t, col_out, l);
        st.col_chunk = cptr != nullptr ? LF(int, col_idx, l) / 16 : -1;
        st.rc = __builtin_amdgcn_make_buffer_rsrc(cptr, 0, cptr ? c.M * 4 : 0, RSRC_W3);
        st.n1 = NC;
    } else {
        float* o2 = LF(fptr_t, out2, l);
        st.n1 = o2 != nullptr ? 2 * LF(int, n1, l) : NC;
        const int ldo2 = o2 != nullptr ? (int)LF(int64_t, ldo2, l) : 0;
        st.colok2 = ldo2 - 4 * g;
        st.ro2 = __builtin_amdgcn_make_buffer_rsrc(o2, 0, o2 ? c.M * ldo2 * 4 : 0, RSRC_W3);
#pragma unroll
        for (int sb = 0; sb < SB; ++sb)
            st.row_off2[sb] = row_ok[sb] ? (unsigned)sample[sb] * (unsigned)ldo2 * 4u + 16u * g : OOB;
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) {
            const int sa = (c.lane & 8) == 0 ? sample[sb] : sample[sb] - 8;
            const int sbb = sa + 8;
            st.pa2[sb] = sa < c.M ? (unsigned)sa * (unsigned)ldo2 * 4u + 16u * g : OOB;
            st.pb2[sb] = sbb < c.M ? (unsigned)sbb * (unsigned)ldo2 * 4u + 16u * g : OOB;
        }
        const uint8_t* mi = LF(cu8ptr_t, mask_in, l);
        const __amdgpu_buffer_rsrc_t rmi =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(mi), 0, mi != nullptr ? c.M * 32 : 0, RSRC_W3);
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) {
            const unsigned off = st.mrow_off[sb];
            typedef unsigned u2 __attribute__((ext_vector_type(2)));
            const u2 w = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(rmi, off, 0, 0));
            st.mi[sb][0] = w.x;
            st.mi[sb][1] = w.y;
            st.mcur[sb] = w.x;
        }
    }

    // ---- HBM-fed input blocks (encodings, gradients): lane (s, g) of block kh holds columns
    // 32 kh + 8 g .. +7 of its sample
    bf16x8 hh[KBH > 0 ? KBH : 1][SB], hl[KBH > 0 ? KBH : 1][SB];
    if constexpr (KBH > 0) {
        const int kb0 = LFI(int, seg_kb, 0, l);
#pragma unroll
        for (int kh = 0; kh < KBH; ++kh) {
            const int sg = kh < kb0 ? 0 : 1;            // segment of this block
            const int khl = sg ? kh - kb0 : kh;
            const int gen = sg ? LFI(int, seg_gen, 1, l) : LFI(int, seg_gen, 0, l);
            if (!is_fwd(MODE) && gen >= 3) {       // the fused composite's head / density gradient
                comp_grad_block(c, gen, sg ? LFI(cfptr_t, seg_ptr, 1, l) : LFI(cfptr_t, seg_ptr, 0, l), sample,
                                row_ok, hh[kh], hl[kh]);
                continue;
            }
            if (is_fwd(MODE) && gen != 0) {
                if constexpr (KBR == 0) {               // the first layer: generated at the tile start, still in LDS
#pragma unroll
                    for (int sb = 0; sb < SB; ++sb)
                        gen_block(c, 16 * sb + (c.lane & 15), 32 * khl + 8 * g, hh[kh][sb], hl[kh][sb]);
                } else {                                // a later layer: the block captured at the tile start
#pragma unroll
                    for (int sb = 0; sb < SB; ++sb) {
                        hh[kh][sb] = c.gh[sb];
                        hl[kh][sb] = c.gl[sb];
                    }
                }
                continue;
            }
            const float* p = sg ? LFI(cfptr_t, seg_ptr, 1, l) : LFI(cfptr_t, seg_ptr, 0, l);
            const int64_t ld = sg ? LFI(int64_t, seg_ld, 1, l) : LFI(int64_t, seg_ld, 0, l);
            const int k = sg ? LFI(int, seg_k, 1, l) : LFI(int, seg_k, 0, l);
            const int rd = sg ? LFI(int, seg_rd, 1, l) : LFI(int, seg_rd, 0, l);
            const int rows = sg ? LFI(int, seg_rows, 1, l) : LFI(int, seg_rows, 0, l);
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, (int)((int64_t)rows * ld * 4), RSRC_W3);
            const int col = 32 * khl + 8 * g;
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) {
                const unsigned m = (unsigned)(row_ok[sb] ? sample[sb] : 0);
                const unsigned row = rd == 1 ? m : m / (unsigned)rd;
                const unsigned rbase = (unsigned)(((int64_t)row * ld + col) * 4);
                const f4 x0 = __builtin_amdgcn_raw_buffer_load_b128(rs, col < k ? rbase : OOB, 0, 0);
                const f4 x1 = __builtin_amdgcn_raw_buffer_load_b128(rs, col + 4 < k ? rbase + 16 : OOB, 0, 0);
                split8(__builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7), hh[kh][sb], hl[kh][sb]);
            }
        }
    }
    // the split HBM-fed operand stays in registers for the whole chunk loop: hipcc otherwise keeps
    // the fp32 rows and redoes the split in every chunk (8 conversions + 4 subtracts + 4 shifts per
    // block and chunk: 32-64 VALU per chunk of the skip / head layers)
    if constexpr (KBH > 0) {
#pragma unroll
        for (int kh = 0; kh < KBH; ++kh)
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) {
                if constexpr (is_x1(MODE))
                    asm volatile("" : "+v"(hh[kh][sb]));
                else
                    asm volatile("" : "+v"(hh[kh][sb]), "+v"(hl[kh][sb]));
            }
    }
    const unsigned hbm_frag = (unsigned)LF(int, hbm_off, l) + (unsigned)c.lane * 16u;

    // the previous chunk's accumulators (its epilogue runs during the current chunk)
    f4 pv[SB] = {};
    if constexpr (KBR == 0) {
        // The first layer has no register-fed part and no DMA.  Its weight fragments (and biases)
        // come from L2 one chunk ahead through builtin buffer loads whose waits hipcc counts, so a
        // chunk's MFMAs do not wait for an L2 round trip and the previous chunk's stores are not
        // drained in every chunk (the form below — asm loads waited with vmcnt(0) — paid both in
        // each of the layer's 8-16 chunks).
        typedef bf16x8 fragk_t[KBH > 0 ? KBH : 1][2];
        auto frag_load = [&](fragk_t& f, int ch) __attribute__((always_inline)) {
#pragma unroll
            for (int kh = 0; kh < KBH; ++kh)
#pragma unroll
                for (int hl_ = 0; hl_ < (is_x1(MODE) ? 1 : 2); ++hl_)
                    f[kh][hl_] = __builtin_bit_cast(
                        bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                    c.rimg, hbm_frag + (unsigned)(((ch * KBH + kh) * 2 + hl_) * 1024), 0, 0));
        };
        auto bias_load = [&](int ch) __attribute__((always_inline)) {
            return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                              c.rimg, st.bias_off + (is_fwd(MODE) ? 64u * (unsigned)ch : 0u), 0, 0));
        };
        // two fragment / bias buffers used alternately (a register copy of a just-issued load would
        // wait for it): chunk ch multiplies `cur` while chunk ch + 1's loads land in `nxt`
        fragk_t hA, hB;
        f4 bA, bB = f4{0.f, 0.f, 0.f, 0.f};
        frag_load(hA, 0);
        auto step = [&](int ch, fragk_t& cur, fragk_t& nxt, f4& bthis, const f4& bprev) __attribute__((always_inline)) {
            frag_load(nxt, ch + 1 < NC ? ch + 1 : ch);    // (past the end: a harmless repeat)
            bthis = bias_load(ch);
            f4 a[SB];
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) a[sb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kh = 0; kh < KBH; ++kh) {
                if constexpr (!is_x1(MODE)) {
#pragma unroll
                    for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(cur[kh][1], hh[kh][sb], a[sb]);
#pragma unroll
                    for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(cur[kh][0], hl[kh][sb], a[sb]);
                }
#pragma unroll
                for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(cur[kh][0], hh[kh][sb], a[sb]);
            }
            // the previous chunk's epilogue (all parts: no register-fed stages to place them in)
#pragma unroll
            for (int i = 0; i < EPI_NP; ++i) epi_part<MODE>(c, st, epi_part_of(i), ch - 1, pv, bprev);
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) pv[sb] = a[sb];
        };
        for (int ch = 0; ch < NC; ch += 2) {
            step(ch, hA, hB, bA, bB);
            if (ch + 1 < NC) step(ch + 1, hB, hA, bB, bA);
        }
    } else
    {
    // one chunk; EP: the compile-time parity of its predecessor (whose epilogue it runs)
    auto chunk = [&](int ch, auto ep_tag) __attribute__((always_inline)) {
        constexpr int EP = decltype(ep_tag)::value;
        // the previous chunk's biases (rows 4 g .. 4 g + 3), for its epilogue in this chunk, issued
        // before this chunk's DMA so that waiting for it does not wait for the DMA
        f4 pb = {0.f, 0.f, 0.f, 0.f};
        if constexpr (is_fwd(MODE))
            buf_load16(pb, st.bias_off + 64u * (unsigned)(ch > 0 ? ch - 1 : 0), c.rimg);
        const unsigned sa = lds_addr(c.smem + c.cur * SLOT_BYTES + c.lane * 16);
        bf16x8 fr[FA][2];
        if constexpr (KBR > 0) {
            // this chunk's DMA share has landed (issued at the start of the previous register-fed
            // chunk and followed by >= after_dma_vm vector-memory ops), then everyone else's; the
            // other slot is free
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(after_dma_vm<MODE>()) : "memory");
#ifndef NERF_FUSED_DIAG_NOBARRIER      // diagnostic builds only (timing without the per-chunk barrier)
            barrier();
#endif
#ifdef NERF_FUSED_DIAG_BAR2             // diagnostic builds only: a second barrier (the cost of one at aligned waves)
            barrier();
#endif
            first_reads<MODE, KBR, 0>(fr, sa);
            issue_dma(c, c.cur ^ 1);                 // the next register-fed chunk, a whole chunk ahead
            __builtin_amdgcn_sched_barrier(0);      // keep the DMA ahead of this chunk's vmem ops (vmcnt)
        }
        // this chunk's HBM-fed weight fragments, from L2
        bf16x8 hf[KBH > 0 ? KBH : 1][2];
#pragma unroll
        for (int kh = 0; kh < KBH; ++kh)
#pragma unroll
            for (int hl_ = 0; hl_ < (is_x1(MODE) ? 1 : 2); ++hl_)
                buf_load16(hf[kh][hl_], hbm_frag + (unsigned)(((ch * KBH + kh) * 2 + hl_) * 1024), c.rimg);
        f4 a[SB];
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) a[sb] = f4{0.f, 0.f, 0.f, 0.f};
        reg_steps<MODE, KBR, KBH, 0, EP>(c, st, sa, fr, a, pv, pb, ch);
        // the HBM-fed fragments have landed: with a register-fed part the 4 epilogue stores of parts
        // 0-1 were issued after them
#pragma unroll
        for (int kh = 0; kh < KBH; ++kh) {
            if constexpr (is_x1(MODE))
                frag_vwait1<(KBR > 0 ? 2 * SB : 0)>(hf[kh][0]);
            else
                frag_vwait<(KBR > 0 ? 2 * SB : 0)>(hf[kh][0], hf[kh][1]);
        }
#pragma unroll
        for (int kh = 0; kh < KBH; ++kh) {
            if constexpr (!is_x1(MODE)) {
#pragma unroll
                for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(hf[kh][1], hh[kh][sb], a[sb]);
#pragma unroll
                for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(hf[kh][0], hl[kh][sb], a[sb]);
            }
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) a[sb] = mfma16(hf[kh][0], hh[kh][sb], a[sb]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (KBR == 0) bias_wait<0>(pb);
        // the parts the stages did not take (all of them for the first layer)
#pragma unroll
        for (int i = epi_placed<KBR, EPI0>(); i < EPI_NP; ++i) epi_part<MODE, EP>(c, st, epi_part_of(i), ch - 1, pv, pb);
        if constexpr (KBR > 0) c.cur ^= 1;
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) pv[sb] = a[sb];
    };
    // unrolled by two: chunk ch (even) runs the epilogue of the odd chunk ch - 1 (none for ch = 0:
    // its stores are dropped), chunk ch + 1 that of the even chunk ch — the pair-store parity, the
    // stash and the accumulator hand-over are compile-time, with no branch or register copy per chunk
    for (int ch = 0; ch < NC; ch += 2) {
        chunk(ch, std::integral_constant<int, 1>{});
        if (ch + 1 < NC) chunk(ch + 1, std::integral_constant<int, 0>{});
    }
    }
    {
        f4 lb = {0.f, 0.f, 0.f, 0.f};
        if constexpr (is_fwd(MODE)) {
            buf_load16(lb, st.bias_off + 64u * (unsigned)(NC - 1), c.rimg);
            bias_wait<0>(lb);
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) epi_part<MODE>(c, st, p, NC - 1, pv, lb);
    }
    if constexpr (is_fwd(MODE)) {
        // the lane's two mask words, each chunk's nibble at 4 (7 - (ch & 7)) whatever the chunk count
        const int nb = NC < 2 * KBMAX ? NC : 2 * KBMAX;
        if (nb < 8) {
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) {
                st.mw[sb][0] = st.mw[sb][1] << (4 * (8 - nb));
                st.mw[sb][1] = 0;
            }
        } else if (nb > 8) {
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) st.mw[sb][1] <<= 4 * (16 - nb);
        }
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int sb = 0; sb < SB; ++sb)
            __builtin_amdgcn_raw_buffer_store_b64(u2{st.mw[sb][0], st.mw[sb][1]}, st.rm, st.mrow_off[sb], 0, 0);
    }
    if constexpr (is_fwd(MODE)) {
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) c.head[sb] = pv[sb];
    }
    if (l + 1 == c.n_layers) return;     // (no next layer: the image region may hold the tile's heads)
    // the next layer's operand: the wave's LDS image back into registers (same wave: LDS ops in order)
#pragma unroll
    for (int kb = 0; kb < KBMAX; ++kb)
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) {
            c.xh[kb][sb] = *reinterpret_cast<const bf16x8*>(c.ximg + ((kb * SB + sb) * 2) * 1024 + c.lane * 16);
            c.xl[kb][sb] = *reinterpret_cast<const bf16x8*>(c.ximg + ((kb * SB + sb) * 2 + 1) * 1024 + c.lane * 16);
        }
}

// ---- compositing fused into the forward (nerf_mlp_fused_render): at the end of a tile the waves
// hand their samples' raw heads and interval lengths to the wave compositing each ray, through that
// wave's operand-image region at COMP_OFF.  The last layer (one 16-row chunk) writes only the first
// 2 SB KB of its image and its image is not read back; every wave passed that layer's chunk barrier
// after reading back its previous image, and a region is next written by its own wave (the next
// tile's generated rows, then its first layer) after it has composited: one barrier suffices.
// A ray of 256 samples spans two tiles, which one workgroup runs back to back (the tile loop walks
// tile pairs): after the first the waves keep their samples' heads and interval lengths in
// registers; after the second they hand both halves to wave 0, which composites the ray (4 samples
// per lane) with the same routine.  Scratch layout: heads [s] 16 B at 0, interval lengths [s] at
// COMP_DEL.
constexpr int COMP_OFF = 8192;
constexpr int COMP_SMAX = 2 * TILE;
constexpr int COMP_DEL = COMP_SMAX * 16;
static_assert(COMP_OFF >= SB * 2048 && COMP_OFF + COMP_SMAX * 20 <= XIMG_BYTES, "composite scratch");

template <int R, class CT>
__device__ __forceinline__ void composite_wave(CT& c, int64_t ray, int S, int roff = 0) {
    const char* reg = c.ximg + COMP_OFF + roff;
    float rd[R], del[R], rc[R][3];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = r * 64 + c.lane;
        rd[r] = 0.f; del[r] = 0.f;
        rc[r][0] = rc[r][1] = rc[r][2] = 0.f;
        if (s < S) {
            const f4 h = *reinterpret_cast<const f4*>(reg + s * 16);
            rc[r][0] = h[0]; rc[r][1] = h[1]; rc[r][2] = h[2]; rd[r] = h[3];
            del[r] = *reinterpret_cast<const float*>(reg + COMP_DEL + s * 4);
        }
    }
    float w[R], rgb[3], cc[R][3], cs[R][3];
    composite_ray<R, true>(S, CF(float, scale_a), CF(float, scale_b), 1, CF(float, density_shift), c.lane, rd, del,
                           rc, w, rgb, cc, cs);
    const int64_t base = ray * S;
    float* wo = CF(fptr_t, weights);
    float* co = CF(fptr_t, coef);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = r * 64 + c.lane;
        if (s < S) {
            // nontemporal (the next tile's first chunk waits for every store's acknowledgement)
            if (wo != nullptr) __builtin_nontemporal_store(w[r], wo + base + s);
            if (co != nullptr) {
                f4* q = reinterpret_cast<f4*>(co + (base + s) * 8);
                __builtin_nontemporal_store(f4{cc[r][0], cc[r][1], cc[r][2], 0.f}, q);
                __builtin_nontemporal_store(f4{cs[r][0], cs[r][1], cs[r][2], 0.f}, q + 1);
            }
        }
    }
    if (c.lane == 0) {
        float* o = CF(fptr_t, rgb) + ray * 3;
        __builtin_nontemporal_store(rgb[0], o);
        __builtin_nontemporal_store(rgb[1], o + 1);
        __builtin_nontemporal_store(rgb[2], o + 2);
    }
}

__device__ __forceinline__ void composite_tile(Ctx& c, int tile) {
#ifdef NERF_FUSED_DIAG_NOCOMP          // diagnostic builds only: timing without the tile-end compositing
    return;
#endif
    const int S = CF(int32_t, samples_per_ray);
    const bool col_sigma = CF(int32_t, sigma_layer) >= 0;
    if (S > TILE) {
        // S = 2 TILE: the ray of tiles (2 q, 2 q + 1); M % S == 0, so every sample is valid
        if ((tile & 1) == 0) {
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) {
                c.phead[sb] = c.head[sb];
                if (col_sigma) c.phead[sb][3] = c.sig[sb];
                c.pcdist[sb] = c.cdist[sb];
            }
            return;
        }
        if (c.lane < 16) {
            char* reg = c.smem + NSLOT * SLOT_BYTES + COMP_OFF;    // wave 0's region
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) {
                const int j = c.wave * SPW + 16 * sb + c.lane;
                f4 h = c.head[sb];
                if (col_sigma) h[3] = c.sig[sb];
                *reinterpret_cast<f4*>(reg + j * 16) = c.phead[sb];
                *reinterpret_cast<float*>(reg + COMP_DEL + j * 4) = c.pcdist[sb];
                *reinterpret_cast<f4*>(reg + (TILE + j) * 16) = h;
                *reinterpret_cast<float*>(reg + COMP_DEL + (TILE + j) * 4) = c.cdist[sb];
            }
        }
        barrier();
        asm volatile("" ::: "memory");
        if (c.wave == 0) composite_wave<(2 * TILE) / 64>(c, (int64_t)(tile >> 1), S);
        return;
    }
    if (c.lane < 16) {
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) {
            const int j = c.wave * SPW + 16 * sb + c.lane;       // sample of the tile
            if (tile * TILE + j < c.M) {
                const int r = j / S, o = j - r * S;
                char* reg = c.smem + NSLOT * SLOT_BYTES + r * XIMG_BYTES + COMP_OFF;
                f4 h = c.head[sb];
                if (col_sigma) h[3] = c.sig[sb];
                *reinterpret_cast<f4*>(reg + o * 16) = h;
                *reinterpret_cast<float*>(reg + COMP_DEL + o * 4) = c.cdist[sb];
            }
        }
    }
    barrier();
    // (s_barrier is no memory operation to the compiler: without this clobber the scratch reads
    // below may be hoisted above it, before the other waves' writes have landed)
    asm volatile("" ::: "memory");
    const int rpt = TILE / S;
    const int64_t ray = (int64_t)tile * rpt + c.wave;
    if (c.wave < rpt && ray * S < c.M) {
        if (S > 64)
            composite_wave<2>(c, ray, S);
        else
            composite_wave<1>(c, ray, S);
    }
}

template <int MODE>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(NWAVE / 4, NWAVE / 4))) void mlp_fused_kernel(FusedArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT_BYTES + NWAVE * XIMG_BYTES];
    Ctx c;
    c.kargs = (kchar_t*)__builtin_amdgcn_kernarg_segment_ptr();
    c.smem = smem;
    c.rimg = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(a.img), 0, a.img_bytes, RSRC_W3);
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.ximg = smem + NSLOT * SLOT_BYTES + c.wave * XIMG_BYTES;
    c.lane = threadIdx.x & 63;
    c.M = a.M;
    c.n_layers = a.n_layers;
    c.dsink = 0.f;
    if ((int)blockIdx.x >= a.ntiles) return;
    const int ngroups = a.ntiles / a.span;
    const int my_tiles = a.span * ((ngroups - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x);
    int per_tile = 0;
    for (int l = 0; l < a.n_layers; ++l)
        if (dma_units(c, l) > 0) per_tile += n16_of(LF(int, N, l));
    c.d_remaining = my_tiles * per_tile;
    {
        const int l = c.lane < c.n_layers ? c.lane : 0;
        c.t_off = (int)LF(int64_t, img_off, l);
        c.t_units = dma_units(c, l);
        c.t_n16 = n16_of(LF(int, N, l));
        c.t_next = next_ring_layer(c, l + 1 == c.n_layers ? 0 : l + 1);
    }
    const int l0 = next_ring_layer(c, 0);
    if (l0 >= 0) dma_seek(c, l0);
    c.cur = 0;
    if (l0 >= 0) issue_dma(c, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the first chunk (the steady-state wait assumes predecessors)
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < KBMAX; ++kb)
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) {
            c.xh[kb][sb] = bf16x8{};
            c.xl[kb][sb] = bf16x8{};
        }
#pragma unroll
    for (int sb = 0; sb < SB; ++sb) {
        c.gh[sb] = bf16x8{};
        c.gl[sb] = bf16x8{};
    }
    // tile groups of `span` consecutive tiles (one group: one tile, unless rays span two)
    const int span_log = a.span >> 1;                 // span 1 or 2
    auto tile_of = [&](int it) { return (((int)blockIdx.x + (it >> span_log) * (int)gridDim.x) << span_log) + (it & span_log); };
    // the encodings' inputs of the next tile, loaded at the start of this tile's second-to-last layer
    // (their memory round trip no longer opens every tile; at the last / third-to-last layer or before
    // the compositing measured slower, profiles/r05ao)
    float gv0[9], gv1[9];
    if (is_fwd(MODE) && a.gen_mask != 0 && my_tiles > 0) {
        const int nb = tile_of(0) * TILE + c.wave * SPW;
        if (a.gen_mask & 1) gen_load<SPW>(c, 0, nb, gv0);
        if (a.gen_mask & 2) gen_load<SPW>(c, 1, nb, gv1);
    }
    for (int it = 0; it < my_tiles; ++it) {
        const int tile = tile_of(it);
        const int base = tile * TILE + c.wave * SPW;
        if (is_fwd(MODE) && a.comp_on) {
            // the samples' interval lengths for the tile-end compositing (long landed by then)
            const float* dist = CF(cfptr_t, dist);
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) {
                const int m = base + 16 * sb + (c.lane & 15);
                c.cdist[sb] = c.lane < 16 && m < c.M ? dist[m] : 0.f;
            }
        }
#ifndef NERF_FUSED_DIAG_NOGEN           // diagnostic builds only: timing without the tile-start encodings
        if (is_fwd(MODE) && a.gen_mask != 0) {
#else
        if (false) {
#endif
            // the tile's in-kernel encodings (one code copy for every layer type): the inputs of both
            // loaded together, then each into the wave's LDS scratch and out to its HBM rows; the one
            // the first layer reads last, so that its rows are still in LDS
            float v0[9], v1[9];
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                v0[j] = gv0[j];
                v1[j] = gv1[j];
            }
#ifdef NERF_FUSED_DIAG_GEN2             // diagnostic builds only: the encodings twice (same outputs)
#pragma nounroll
            for (int i = 0; i < 4; ++i) {
                const int e = a.gen_lds == 0 ? 1 - (i & 1) : (i & 1);
#else
#pragma nounroll
            for (int i = 0; i < 2; ++i) {
                const int e = a.gen_lds == 0 ? 1 - i : i;
#endif
                if ((a.gen_mask >> e) & 1) {
                    float v[9];
#pragma unroll
                    for (int j = 0; j < 9; ++j) v[j] = e == 0 ? v0[j] : v1[j];
                    gen_rows_lds<SPW>(c, e, base, v);
                    if (e == a.gen_reg) {
                        // the later layer's block from the wave's own rows (same wave: LDS in order)
#pragma unroll
                        for (int sb = 0; sb < SB; ++sb)
                            gen_block(c, 16 * sb + (c.lane & 15), 8 * (c.lane >> 4), c.gh[sb], c.gl[sb]);
                    }
                    gen_store<SPW>(c, e, base);
                }
            }
        }
        for (int l = 0; l < a.n_layers; ++l) {
            if (is_fwd(MODE) && a.gen_mask != 0 && it + 1 < my_tiles &&
                l == (a.n_layers > 2 ? a.n_layers - 2 : 0)) {
                const int nb = tile_of(it + 1) * TILE + c.wave * SPW;
                if (a.gen_mask & 1) gen_load<SPW>(c, 0, nb, gv0);
                if (a.gen_mask & 2) gen_load<SPW>(c, 1, nb, gv1);
            }
            switch (LF(int, type, l)) {
                case 1: fused_layer<MODE, 0, 1>(c, l, base); break;
                case 2: fused_layer<MODE, 0, 2>(c, l, base); break;
                case 3: fused_layer<MODE, 4, 0>(c, l, base); break;
                case 6: fused_layer<MODE, 8, 0>(c, l, base); break;
                case 7: fused_layer<MODE, 8, 1>(c, l, base); break;
                case 8: fused_layer<MODE, 8, 2>(c, l, base); break;
                default: break;                          // rejected on the host
            }
        }
        if (is_fwd(MODE) && a.comp_on) composite_tile(c, tile);
#ifdef NERF_FUSED_DIAG_COMP2            // diagnostic builds only: the compositing twice (same outputs, its cost at unchanged data)
        if (is_fwd(MODE) && a.comp_on) composite_tile(c, tile);
#endif
    }
#ifdef NERF_FUSED_DIAG_MFMAONLY
    if (c.dsink == 1234.5f) LF(fptr_t, out, 0)[threadIdx.x] = c.dsink;   // keeps the MFMAs live
#endif
}
#undef LF
#undef LFI
#undef EF
#undef CF
#undef HG

struct PackArgs {
    const float* src[NERF_FUSED_MAX_SRCS];
};

__global__ __launch_bounds__(256) void fused_pack_kernel(PackArgs p, const int32_t* __restrict__ map_src,
                                                         const int32_t* __restrict__ map_dst, int64_t n,
                                                         char* __restrict__ img) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int s = map_src[i];
    float v = 0.f;
    if (s >= 0) {
        // per-lane index into the by-value pointer table: read it from the kernarg segment
        typedef __attribute__((address_space(4))) const float* const kptr_t;
        kptr_t* tab = (kptr_t*)((kchar_t*)__builtin_amdgcn_kernarg_segment_ptr() + offsetof(PackArgs, src));
        v = tab[s >> 24][s & 0xffffff];
    }
    const int d = map_dst[i];
    if (d >= 0) {
        const __bf16 hi = (__bf16)v;
        const __bf16 lo = (__bf16)(v - (float)hi);
        __bf16* b = reinterpret_cast<__bf16*>(img);
        b[d] = hi;
        b[d + 512] = lo;
    } else {
        reinterpret_cast<float*>(img)[~d] = v;
    }
}

int num_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

}  // namespace

namespace {
int enc_out_dim(const nerf_pe_params& p) { return (2 * p.levels + (p.include_identity ? 1 : 0)) * 3; }

// a generated segment's encoding, checked as nerf_encode_fwd checks its arguments
bool hash_ok(const nerf_fused_encoding& e) {
    const nerf_hashgrid_params* h = e.hash;
    if (h == nullptr || e.hash_table == nullptr || !aligned16(e.hash_table)) return false;
    if (h->levels < 1 || h->levels > 16 || !(h->features == 1 || h->features == 2 || h->features == 4)) return false;
    if (h->table_size < 1 || (int64_t)h->levels * h->table_size * h->features >= ((int64_t)1 << 31)) return false;
    if (!(h->normalize == 0 || h->normalize == 1) || !(h->query == 0 || h->query == 1)) return false;
    if (e.params.query != h->query || e.per_ray || e.out_dim != h->levels * h->features) return false;
    for (int l = 0; l < h->levels; ++l)
        if (h->res[l] < 1 || h->res[l] > (1 << 20)) return false;
    return true;
}

bool encoding_ok(const nerf_fused_encoding& e, int64_t M) {
    const nerf_pe_params& p = e.params;
    if (p.kind == 2) {
        if (!hash_ok(e)) return false;
    } else if (!(p.levels >= 0 && p.levels <= 16 && (p.kind == 0 || p.kind == 1))) {
        return false;
    }
    if ((p.kind != 2 && e.out_dim != enc_out_dim(p)) || e.out_dim <= 0 || e.samples_per_ray < 1 || e.n_rays < 1)
        return false;
    if (e.n_rays * e.samples_per_ray < M || M >= ((int64_t)1 << 31)) return false;
    if (e.ray_d == nullptr) return false;
    if (e.per_ray) {
        if (p.kind != 0) return false;                       // nerf_encode_rays: plain Fourier features
    } else {
        if (e.ray_o == nullptr || e.t_start == nullptr || (p.query != 0 && e.t_end == nullptr)) return false;
        if (p.kind == 1 && (e.t_end == nullptr || e.pixel_width == nullptr || p.pw_mode < 0 || p.pw_mode > 2))
            return false;
    }
    if (e.out != nullptr) {
        const int64_t rows = e.per_ray ? e.n_rays : M;
        if (!aligned16(e.out) || e.ld % 4 != 0 || e.ld < e.out_dim || rows * e.ld * 4 >= ((int64_t)1 << 31))
            return false;
    }
    return true;
}
}  // namespace

namespace {
int fused_launch(const nerf_fused_layer* layers, int32_t n_layers, const void* image, int64_t M,
                 const nerf_fused_encoding* encodings, const nerf_fused_composite* comp, int32_t flags, void* stream) {
    NERF_REQUIRE((flags & ~NERF_FUSED_BF16) == 0);
    const bool single_pass = (flags & NERF_FUSED_BF16) != 0;
    NERF_REQUIRE(layers != nullptr && image != nullptr);
    NERF_REQUIRE(n_layers >= 1 && n_layers <= NERF_FUSED_MAX_LAYERS);
    NERF_REQUIRE(M >= 1 && M <= (int64_t)1 << 30);
    FusedArgs a;
    int64_t img_end = 0;
    int gen_lds = -1, gen_reg = -1;
    // the input-gradient chain (a layer multiplies by ReLU bits or routes rows to a second output):
    // no bias, no ReLU, no mask bits or column outputs; otherwise the forward, which has none of those
    bool dgrad = false;
    for (int l = 0; l < n_layers; ++l) dgrad = dgrad || layers[l].mask_in != nullptr || layers[l].out2 != nullptr;
    for (int l = 0; l < n_layers; ++l) {
        if (dgrad)
            NERF_REQUIRE(layers[l].relu == 0 && layers[l].mask == nullptr && layers[l].col_out == nullptr);
    }
    for (int l = 0; l < n_layers; ++l) {
        const nerf_fused_layer& L = layers[l];
        const int kbr = (L.type / 3) * 4, kbh = L.type % 3;
        NERF_REQUIRE(L.type == 1 || L.type == 2 || L.type == 3 || L.type == 6 || L.type == 7 || L.type == 8);
        NERF_REQUIRE((l == 0) == (kbr == 0));                  // only the first layer has no register input
        NERF_REQUIRE(L.N >= 1 && L.nb == (L.N + 31) / 32 && L.nb <= 16);
        const int n16 = (L.N + 15) / 16;
        NERF_REQUIRE(L.chunk_units == 2 * kbr);
        NERF_REQUIRE(L.img_off >= 0 && L.img_off % 1024 == 0);
        NERF_REQUIRE(L.hbm_off >= 0 && L.hbm_off % 1024 == 0);
        NERF_REQUIRE(L.bias_off >= 0 && L.bias_off % 16 == 0);
        img_end = img_end > L.img_off + (int64_t)n16 * 2048 * kbr ? img_end : L.img_off + (int64_t)n16 * 2048 * kbr;
        img_end = img_end > (int64_t)L.hbm_off + (int64_t)n16 * 2048 * kbh ? img_end
                                                                          : (int64_t)L.hbm_off + (int64_t)n16 * 2048 * kbh;
        img_end = img_end > L.bias_off + 64 * n16 ? img_end : L.bias_off + 64 * n16;
        // with a second output only the first n1 32-column chunks land in out (columns past ldo are
        // dropped); a null out (ldo 0) drops the layer's stores (inference keeps only the exposed outputs)
        NERF_REQUIRE((L.out == nullptr && L.ldo == 0) ||
                     (L.out != nullptr && aligned16(L.out) && L.ldo % 4 == 0 &&
                      L.ldo >= (L.out2 != nullptr ? (32 * L.n1 < L.N ? 32 * L.n1 : L.N) : L.N)));
        NERF_REQUIRE(M * L.ldo * 4 < ((int64_t)1 << 31));
        NERF_REQUIRE(L.mask == nullptr || (L.N <= 256 && M * 32 < ((int64_t)1 << 31)));
        NERF_REQUIRE(L.mask_in == nullptr || M * 32 < ((int64_t)1 << 31));
        NERF_REQUIRE(L.col_out == nullptr || (L.col_idx >= 0 && L.col_idx % 32 == 0 && L.col_idx < L.N));
        NERF_REQUIRE(L.out2 == nullptr || (aligned16(L.out2) && L.ldo2 % 4 == 0 && L.ldo2 > 0 && L.n1 >= 0 &&
                                           L.n1 <= L.nb && M * L.ldo2 * 4 < ((int64_t)1 << 31)));
        NERF_REQUIRE(L.nseg >= 0 && L.nseg <= 2);
        int kbs = 0;
        for (int s = 0; s < 2; ++s) {
            const int gen = s < L.nseg ? L.seg_gen[s] : 0;
            NERF_REQUIRE(s < L.nseg || L.seg_gen[s] == 0);
            if (gen == 0) continue;
            if (gen >= 3) {
                // the fused composite's gradient rows (input-gradient chain): one coefficient block
                NERF_REQUIRE(dgrad && gen <= 4 && comp != nullptr && comp->grad_rgb != nullptr && L.nseg == 1);
                NERF_REQUIRE(L.seg_kb[0] == 1 && L.seg_k[0] == 8 && L.seg_ld[0] == 8 && L.seg_rd[0] == 1);
                NERF_REQUIRE(L.seg_ptr[0] != nullptr && aligned16(L.seg_ptr[0]) && L.seg_rows[0] >= M);
                NERF_REQUIRE((int64_t)L.seg_rows[0] * 32 < ((int64_t)1 << 31));
                float* o = gen == 3 ? comp->grad_head : comp->grad_sigma;
                const int64_t ld = gen == 3 ? comp->ld_head : comp->ld_sigma;
                NERF_REQUIRE(o == nullptr || (aligned16(o) && ld % 4 == 0 && ld >= 4));
                const int S = comp->samples_per_ray;
                NERF_REQUIRE(S >= 1 && M % S == 0);
                continue;
            }
            // rows generated at the tile start: the first layer reads them from LDS (one segment); a
            // later layer reads one k-block of them from the registers captured at the tile start
            NERF_REQUIRE(!dgrad && encodings != nullptr && (gen == 1 || gen == 2));
            const nerf_fused_encoding& e = encodings[gen - 1];
            NERF_REQUIRE(e.out_dim > 0 && e.out_dim <= 32 * L.seg_kb[s] && 32 * L.seg_kb[s] <= 64);
            if (l == 0) {
                NERF_REQUIRE(gen_lds < 0);
                gen_lds = gen - 1;
            } else {
                NERF_REQUIRE(L.seg_kb[s] == 1 && (gen_reg < 0 || gen_reg == gen - 1));
                gen_reg = gen - 1;
            }
        }
        for (int s = 0; s < L.nseg; ++s) {
            kbs += L.seg_kb[s];
            if (L.seg_gen[s] != 0) continue;
            NERF_REQUIRE(L.seg_ptr[s] != nullptr && aligned16(L.seg_ptr[s]));
            NERF_REQUIRE(L.seg_k[s] % 4 == 0 && L.seg_k[s] <= 32 * L.seg_kb[s] && L.seg_ld[s] % 4 == 0);
            NERF_REQUIRE(L.seg_ld[s] >= L.seg_k[s] && L.seg_rd[s] >= 1 && L.seg_rows[s] >= (M + L.seg_rd[s] - 1) / L.seg_rd[s]);
            NERF_REQUIRE((int64_t)L.seg_rows[s] * L.seg_ld[s] * 4 < ((int64_t)1 << 31));
        }
        NERF_REQUIRE(kbs == kbh);
        if (l > 0) {
            // the fed k-blocks are complete 32-row blocks of the previous layer's fed output
            const nerf_fused_layer& P = layers[l - 1];
            NERF_REQUIRE(32 * kbr <= (P.out2 != nullptr ? 32 * P.n1 : P.N));
        }
        a.L[l] = L;
        if (L.nseg < 2) {
            a.L[l].seg_kb[1] = 0;
            a.L[l].seg_ptr[1] = L.nseg == 1 ? L.seg_ptr[0] : nullptr;
            a.L[l].seg_gen[1] = 0;
        }
        if (L.nseg < 1) a.L[l].seg_gen[0] = 0;
    }
    NERF_REQUIRE(img_end < ((int64_t)1 << 31));
    // generated encodings (out_dim > 0): checked as nerf_encode_fwd checks its arguments; their rows
    // are always stored (later layers and the weight gradients read them)
    int gen_mask = 0;
    memset(&a.hg, 0, sizeof(a.hg));
    a.hg_table = nullptr;
    memset(a.hg_off, 0, sizeof(a.hg_off));
    for (int e = 0; e < 2; ++e) {
        if (encodings != nullptr && encodings[e].out_dim > 0) {
            NERF_REQUIRE(!dgrad && encoding_ok(encodings[e], M) && encodings[e].out != nullptr && encodings[e].ld <= 64);
            a.enc[e] = encodings[e];
            gen_mask |= 1 << e;
            if (encodings[e].params.kind == 2) {
                // one hash grid per launch: its parameters and level row offsets by value
                NERF_REQUIRE(a.hg_table == nullptr);
                a.hg = *encodings[e].hash;
                a.hg_table = encodings[e].hash_table;
                int64_t off = 0;
                for (int l = 0; l < a.hg.levels; ++l) {
                    a.hg_off[l] = (int)off;
                    off += level_rows(a.hg.res[l], a.hg.table_size);
                }
            }
        } else {
            memset(&a.enc[e], 0, sizeof(a.enc[e]));
        }
    }
    NERF_REQUIRE(gen_lds < 0 || ((gen_mask >> gen_lds) & 1));
    NERF_REQUIRE(gen_reg < 0 || ((gen_mask >> gen_reg) & 1));
    // Ordering rule for generated rows read back from HBM inside the launch (seg_gen 0 with seg_ptr in
    // a generated encoding's rows): only the wave that stored a row may read it (one wave's vector
    // memory operations complete in order through the CU's L1), i.e. per-sample rows (not per_ray)
    // read at row divisor 1.  A per-ray row is stored once, by the wave holding the ray's first
    // sample — possibly another workgroup of the grid, with no ordering — so a later layer must take
    // a per-ray encoding from the tile-start registers (seg_gen) or the caller fills it beforehand.
    for (int l = 0; l < n_layers && gen_mask != 0; ++l) {
        const nerf_fused_layer& L = layers[l];
        for (int s = 0; s < L.nseg; ++s) {
            if (L.seg_gen[s] != 0) continue;
            const char* p = static_cast<const char*>(static_cast<const void*>(L.seg_ptr[s]));
            const char* pe = p + (int64_t)L.seg_rows[s] * L.seg_ld[s] * 4;
            for (int e = 0; e < 2; ++e) {
                if (!((gen_mask >> e) & 1)) continue;
                const nerf_fused_encoding& E = encodings[e];
                const char* q = static_cast<const char*>(static_cast<const void*>(E.out));
                const char* qe = q + (E.per_ray ? E.n_rays : M) * E.ld * 4;
                if (p < qe && q < pe)
                    NERF_REQUIRE((!E.per_ray || E.samples_per_ray == 1) && L.seg_rd[s] == 1 && p == q && L.seg_ld[s] == E.ld);
            }
        }
    }
    a.gen_mask = gen_mask;
    a.gen_lds = gen_lds;
    a.gen_reg = gen_reg;
    a.img = static_cast<const char*>(image);
    a.img_bytes = (int)img_end;
    a.n_layers = n_layers;
    a.M = (int)M;
    a.ntiles = (int)((M + TILE - 1) / TILE);
    a.span = 1;
    // compositing fused into the forward (include/nerf_amd.h nerf_fused_composite)
    a.comp_on = 0;
    memset(&a.comp, 0, sizeof(a.comp));
    if (comp != nullptr) {
        a.comp = *comp;
        const int S = comp->samples_per_ray;
        if (!dgrad) {
            NERF_REQUIRE(((S >= 16 && S <= TILE && TILE % S == 0 && TILE / S <= NWAVE) || S == 2 * TILE) &&
                         M % S == 0);
            if (S == 2 * TILE) a.span = 2;
            NERF_REQUIRE(comp->dist != nullptr && comp->rgb != nullptr);
            NERF_REQUIRE(comp->coef == nullptr || (aligned16(comp->coef) && M * 32 < ((int64_t)1 << 31)));
            // the heads: the last layer, one 16-row chunk with a barrier (a register-fed part)
            const nerf_fused_layer& H = layers[n_layers - 1];
            NERF_REQUIRE(comp->head_layer == n_layers - 1 && H.type >= 3 && H.N <= 16);
            NERF_REQUIRE(H.N >= (comp->sigma_layer < 0 ? 4 : 3));
            NERF_REQUIRE(comp->sigma_layer < n_layers - 1);
            if (comp->sigma_layer >= 0) NERF_REQUIRE(layers[comp->sigma_layer].col_out != nullptr);
            a.comp_on = 1;
        }
    }
    const int ngroups = a.ntiles / a.span;
    const int grid = ngroups < num_cus() ? ngroups : num_cus();
    if (single_pass) {
        if (dgrad)
            hipLaunchKernelGGL(mlp_fused_kernel<MODE_DGRAD | MODE_X1>, dim3(grid), dim3(WG), 0, as_stream(stream), a);
        else
            hipLaunchKernelGGL(mlp_fused_kernel<MODE_FWD | MODE_X1>, dim3(grid), dim3(WG), 0, as_stream(stream), a);
    } else if (dgrad) {
        hipLaunchKernelGGL(mlp_fused_kernel<MODE_DGRAD>, dim3(grid), dim3(WG), 0, as_stream(stream), a);
    } else {
        hipLaunchKernelGGL(mlp_fused_kernel<MODE_FWD>, dim3(grid), dim3(WG), 0, as_stream(stream), a);
    }
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
}  // namespace

extern "C" int nerf_mlp_fused_fwd(const nerf_fused_layer* layers, int32_t n_layers, const void* image, int64_t M,
                                  const nerf_fused_encoding* encodings, void* stream) {
    return fused_launch(layers, n_layers, image, M, encodings, nullptr, 0, stream);
}

extern "C" int nerf_mlp_fused_render(const nerf_fused_layer* layers, int32_t n_layers, const void* image, int64_t M,
                                     const nerf_fused_encoding* encodings, const nerf_fused_composite* composite,
                                     void* stream) {
    return fused_launch(layers, n_layers, image, M, encodings, composite, 0, stream);
}

extern "C" int nerf_mlp_fused_run(const nerf_fused_layer* layers, int32_t n_layers, const void* image, int64_t M,
                                  const nerf_fused_encoding* encodings, const nerf_fused_composite* composite,
                                  int32_t flags, void* stream) {
    return fused_launch(layers, n_layers, image, M, encodings, composite, flags, stream);
}

extern "C" int nerf_fused_pack(const float* const* srcs, int32_t n_srcs, const int32_t* map_src,
                               const int32_t* map_dst, int64_t n, void* image, void* stream) {
    NERF_REQUIRE(srcs != nullptr && map_src != nullptr && map_dst != nullptr && image != nullptr);
    NERF_REQUIRE(n_srcs >= 1 && n_srcs <= NERF_FUSED_MAX_SRCS && n >= 0);
    if (n == 0) return NERF_OK;
    PackArgs p;
    for (int i = 0; i < NERF_FUSED_MAX_SRCS; ++i) p.src[i] = i < n_srcs ? srcs[i] : nullptr;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(fused_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), p, map_src,
                       map_dst, n, static_cast<char*>(image));
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" __attribute__((visibility("hidden"))) int32_t nerf_tu_build_flags_mlp_fused(void) {
    return NERF_TU_BUILD_FLAGS;
}
