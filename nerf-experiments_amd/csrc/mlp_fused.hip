// Fused field-MLP forward: every Linear (+ bias + ReLU) of a NerfModel in ONE launch
// (a7, barf/model_interpolation_architecture.py:96-141; contract in include/nerf_amd.h).
//
// Layer-by-layer GEMMs move each 256-wide fp32 activation through HBM twice (written by
// one launch, read by the next: 536 MB per layer at 262 144 samples).  Here a wave owns 16
// samples and keeps their activations in registers across the whole network:
//
//   out^T[n][s] = W[n][:] . x^T[:][s]    A operand = weights (rows n), B = activations (cols s)
//
// on v_mfma_f32_16x16x32_bf16.  Its 16x16 accumulator holds, in lane (s, g) (s = lane & 15,
// g = lane >> 4), output rows 4g .. 4g+3 of sample s.  Two such blocks (rows 32q .. 32q+15 and
// 32q+16 .. 32q+31) give lane (s, g) exactly the eight k-values it must supply as the B operand
// of one 32-deep k-block of the next layer, once the reduction index is permuted the same way
// in the packed weights (element j of lane group g <-> feature 32q + 16(j >> 2) + 4g + (j & 3)).
// A layer's output so becomes the next layer's input with no data movement: bias + ReLU + the
// bf16 hi/lo split (3 x bf16 products, as linear_x3.hip) are applied in registers.
//
// Weights (2.6 MB for NerfModel) stream through LDS.  Chunk = 32 output rows of one layer: for
// every k-block the two 16-row A fragments ([hi 64 lanes x 16 B][lo 64 lanes x 16 B] each, one
// conflict-free ds_read_b128 per half) + 1 KB holding the 32 biases.  Chunks are LDS-DMA'd
// (global_load_lds_dwordx4) into a 3-slot ring two chunks ahead and shared by the 8 waves of a
// workgroup (two per SIMD, <= 256 registers each), so the weights cross L2 -> LDS once per
// 128 samples.  Only HBM-fed inputs (encodings) are loaded and only what the backward needs
// (each layer's output, its ReLU mask bits, the density column) is stored.
#include <stddef.h>

#include "common.h"

using namespace nerf;

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

constexpr int SLOT_BYTES = 40 * 1024;      // largest chunk: 10 k-blocks x 4 KB
constexpr int NSLOT = 2;
constexpr int XO_BYTES = 8 * 2048;         // per wave pair: the next layer's B operand, [kb][hi|lo][lane] 16 B
constexpr int MX_BYTES = 64 * 8;           // per wave pair: mask-word exchange (the high nibbles)
constexpr int BIAS_LDS = 12 * 1024;        // all biases of the network ([layer][nb][32] fp32), copied once
constexpr int WG = 512;                    // 8 waves, two per SIMD (<= 256 registers each)
constexpr int NWAVE = WG / 64;
constexpr int SPW = 16;                    // samples per wave pair
constexpr int TILE = NWAVE / 2 * SPW;      // samples per workgroup tile
constexpr int KBMAX = 8;                   // register-fed 32-deep k-blocks (256 features)
constexpr unsigned OOB = 0x80000000u;      // buffer offset past every num_records: load 0 / drop store
constexpr int RSRC_W3 = 0x00020000;
constexpr int EPI_MIN_VM = 2;

struct FusedArgs {
    nerf_fused_layer L[NERF_FUSED_MAX_LAYERS];
    const char* img;
    int bias_base, bias_bytes;   // the biases' byte range in the image (contiguous, layer order)
    int n_layers;
    int M;
    int ntiles;
};

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

__device__ __forceinline__ f4 mfma16(bf16x8 a, bf16x8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// acc += a*b, both operands split hi/lo; small terms first (as linear_x3.hip)
__device__ __forceinline__ f4 mfma_x3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f4 c) {
    c = mfma16(al, bh, c);
    c = mfma16(ah, bl, c);
    return mfma16(ah, bh, c);
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

struct Ctx {
    kchar_t* kargs;
    char* smem;
    const char* img;
    int wave, lane, M, n_layers, bias_base;
    int half;             // which 16-row block of every 32-row chunk this wave computes
    int cur;              // ring slot of the chunk being computed
    // vector-memory ops issued after the newest chunk DMA (= the chunk about to be computed), so
    // s_waitcnt vmcnt(after_last) is exactly its wait
    int after_prev, after_last;
    // DMA cursor: chunks of consecutive layers are contiguous in the image and the stream
    // repeats per tile, so the next chunk is d_off; layer fields are only read when it changes
    int d_off, d_units, d_left, d_layer;
    int d_remaining;      // chunks still to issue
    char* xo;             // the wave pair's LDS image of the next layer's B operand
    char* mx;             // the wave pair's mask-word exchange
    const char* bias;     // LDS copy of the biases
    // the current layer's register-fed input (B operand)
    bf16x8 xh[KBMAX], xl[KBMAX];
};

__device__ __forceinline__ void count_vm(Ctx& c, int n) {
    c.after_prev += n;
    c.after_last += n;
}

// LDS-DMA of the next chunk of the stream into ring slot `slot` (the 8 waves share its 1 KB units)
__device__ __forceinline__ void issue_dma(Ctx& c, int slot) {
    int cnt = 0;
    if (c.d_remaining > 0) {
        const char* src = c.img + c.d_off + c.lane * 16;
        char* dst = c.smem + slot * SLOT_BYTES;
        for (int u = c.wave; u < c.d_units; u += NWAVE) {
            __builtin_amdgcn_global_load_lds((glb_void_t*)(src + u * 1024), (lds_void_t*)(dst + u * 1024), 16, 0, 0);
            ++cnt;
        }
        c.d_off += c.d_units * 1024;
        if (--c.d_left == 0) {
            if (++c.d_layer == c.n_layers) {
                c.d_layer = 0;
                c.d_off = 0;
            }
            c.d_units = LF(int, chunk_units, c.d_layer);
            c.d_left = LF(int, nb, c.d_layer);
        }
        --c.d_remaining;
    }
    c.after_prev = c.after_last + cnt;
    c.after_last = 0;
}

struct LayerState {
    int NB;
    bool row_ok;
    int floor_i;          // ReLU as an integer max on the fp32 bits: 0, or INT_MIN for no ReLU
    int sample, col_idx;
    unsigned sample_off;  // sample * 4 (OOB past M)
    unsigned row_off;     // byte offset of this lane's sample row (OOB past M)
    int64_t ldo;
    __amdgpu_buffer_rsrc_t ro, rm, rc;
    int bias_lds;         // LDS byte offset of the layer's biases (+128 per chunk; >= 128)
    unsigned mw[2];       // ReLU mask words 2g, 2g + 1 of this lane's sample row (this wave's nibbles)
    int n1;               // chunks routed to out (fed forward, masked); the rest go to out2
    unsigned row_off2;    // byte offset of this lane's sample row in out2 (OOB past M)
    int64_t ldo2;
    __amdgpu_buffer_rsrc_t ro2;
    bool mask_in;         // multiply the output by the ReLU bits min (input-gradient chain)
    unsigned mi[8];       // this lane's sample row of those bits
};

// Epilogue of this wave's block of chunk nbc (output rows 32 nbc + 16 half .. +15, accumulator v):
// bias + ReLU, stores, mask bits and the wave pair's B-operand image.  Straight-line code in
// four parts (absent outputs are buffer stores with out-of-range offsets, which the hardware
// drops), placed in the stages of the next chunk so that its VALU work issues in MFMA shadows.
// nbc = -1 (the call in a layer's first chunk) writes nothing visible.
template <int PART>
__device__ __forceinline__ void chunk_epilogue(Ctx& c, LayerState& st, int nbc, f4& v, unsigned& w) {
    const int g = c.lane >> 4;
    if constexpr (PART == 0) {
        const f4 b = *reinterpret_cast<const f4*>(c.bias + st.bias_lds + 128 * nbc + 64 * c.half + 16 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            v[r] = __builtin_bit_cast(float, max(__builtin_bit_cast(int, v[r] + b[r]), st.floor_i));
        const bool sec = nbc >= st.n1;               // an encoding input's rows (chain: out2)
        if (st.mask_in && !sec) {
            // column 32 nbc + 16 half + 4 g + r: bit 4 half + g of byte (nbc & 3) of word 2 r + (nbc >> 2)
            const int sh = 8 * (nbc & 3) + 4 * c.half + g;
            const bool hi = nbc >= 4;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const unsigned word = hi ? st.mi[2 * r + 1] : st.mi[2 * r];
                v[r] = ((word >> sh) & 1u) ? v[r] : 0.f;
            }
        }
        const int colok = nbc >= 0 ? (int)(sec ? st.ldo2 : st.ldo) : 0;
        const int col = 32 * (sec ? nbc - st.n1 : nbc) + 16 * c.half + 4 * g;
        const unsigned off = (unsigned)col < (unsigned)colok ? (sec ? st.row_off2 : st.row_off) + (unsigned)col * 4u
                                                             : OOB;   // nbc = -1: col < 0
        const unsigned coff = (c.half == 0 && g == 0 && st.col_idx == 32 * nbc) ? st.sample_off : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(v, sec ? st.ro2 : st.ro, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[0]), st.rc, coff, 0, 0);
        count_vm(c, 2);
    } else if constexpr (PART == 1) {
        // NERF_EPI_MASKOUT layout: column 32 nb + 16 bb + 4 g + r is bit 4 bb + g of byte (nb & 3)
        // of word 2 r + (nb >> 2) of the row; lane group g keeps the byte of r = g
        w = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) w |= (v[r] > 0.f ? 1u : 0u) << (8 * r + 4 * c.half + g);
    } else if constexpr (PART == 2) {
        const auto x16 = __builtin_amdgcn_permlane16_swap(w, w, false, false);   // OR with lane ^ 16
        w = x16[0] | x16[1];
        const auto x32 = __builtin_amdgcn_permlane32_swap(w, w, false, false);   // OR with lane ^ 32
        w = x32[0] | x32[1];
        const unsigned byte = ((w >> (8 * g)) & 0xffu) << (8 * (nbc & 3));
        st.mw[0] |= (nbc >= 0 && nbc < 4) ? byte : 0u;
        st.mw[1] |= (nbc >= 4 && nbc < 8) ? byte : 0u;
    } else {
        // the next layer's B operand, k-block nbc: elements j < 4 are block 0 (this pair's
        // half-0 wave), j >= 4 block 1 -> 8 bytes of each lane's 16-byte hi and lo slots
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        const bf16x4 h = __builtin_convertvector(v, bf16x4);
        const bf16x4 lo = __builtin_convertvector(v - __builtin_convertvector(h, f4), bf16x4);
        if (nbc >= 0 && nbc < KBMAX && nbc < st.n1) {
            *reinterpret_cast<bf16x4*>(c.xo + nbc * 2048 + c.lane * 16 + 8 * c.half) = h;
            *reinterpret_cast<bf16x4*>(c.xo + nbc * 2048 + 1024 + c.lane * 16 + 8 * c.half) = lo;
        }
    }
}

// one layer: runtime loop over its 32-row output chunks (this wave: one 16-row block of each);
// k-blocks unrolled (KBR register-fed, KBH HBM-fed).  Reads c.xh/c.xl, leaves the next layer's
// input there.
template <int KBR, int KBH>
__device__ __forceinline__ void fused_layer(Ctx& c, int l, int sample) {
    constexpr int KB = KBR + KBH;
    const int g = c.lane >> 4;
    LayerState st;
    st.NB = LF(int, nb, l);
    st.floor_i = LF(int, relu, l) != 0 ? 0 : (int)0x80000000;
    st.ldo = LF(int64_t, ldo, l);
    st.sample = sample;
    st.row_ok = sample < c.M;
    st.row_off = st.row_ok ? (unsigned)((int64_t)sample * st.ldo * 4) : OOB;
    st.sample_off = st.row_ok ? (unsigned)(sample * 4) : OOB;
    st.mw[0] = st.mw[1] = 0;
    st.ro = __builtin_amdgcn_make_buffer_rsrc(LF(fptr_t, out, l), 0, (int)((int64_t)c.M * st.ldo * 4), RSRC_W3);
    uint8_t* mptr = LF(u8ptr_t, mask, l);
    st.rm = __builtin_amdgcn_make_buffer_rsrc(mptr, 0, mptr != nullptr ? c.M * 32 : 0, RSRC_W3);
    float* cptr = LF(fptr_t, col_out, l);
    st.col_idx = cptr != nullptr ? LF(int, col_idx, l) : -1;
    st.rc = __builtin_amdgcn_make_buffer_rsrc(cptr, 0, cptr ? c.M * 4 : 0, RSRC_W3);
    st.bias_lds = (int)LF(int64_t, bias_off, l) - c.bias_base + 128;
    {
        float* o2 = LF(fptr_t, out2, l);
        st.n1 = o2 != nullptr ? LF(int, n1, l) : st.NB;
        st.ldo2 = o2 != nullptr ? LF(int64_t, ldo2, l) : 0;
        st.ro2 = __builtin_amdgcn_make_buffer_rsrc(o2, 0, o2 ? (int)((int64_t)c.M * st.ldo2 * 4) : 0, RSRC_W3);
        st.row_off2 = st.row_ok ? (unsigned)((int64_t)sample * st.ldo2 * 4) : OOB;
    }
    {
        const uint8_t* mi = LF(cu8ptr_t, mask_in, l);
        st.mask_in = mi != nullptr;
        if (st.mask_in) {
            const __amdgpu_buffer_rsrc_t rmi =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(mi), 0, c.M * 32, RSRC_W3);
            const unsigned off = st.row_ok ? (unsigned)(sample * 32) : OOB;
            typedef unsigned u4 __attribute__((ext_vector_type(4)));
            const u4 w0 = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rmi, off, 0, 0));
            const u4 w1 = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rmi, off + 16, 0, 0));
            st.mi[0] = w0.x; st.mi[1] = w0.y; st.mi[2] = w0.z; st.mi[3] = w0.w;
            st.mi[4] = w1.x; st.mi[5] = w1.y; st.mi[6] = w1.z; st.mi[7] = w1.w;
            count_vm(c, 2);
        }
    }

    // ---- HBM-fed input blocks (encodings): lane (s, g) of block kh holds columns 32 kh + 8 g .. +7
    bf16x8 hh[KBH > 0 ? KBH : 1], hl[KBH > 0 ? KBH : 1];
    if constexpr (KBH > 0) {
        const int kb0 = LFI(int, seg_kb, 0, l);
        f8 raw[KBH];
#pragma unroll
        for (int kh = 0; kh < KBH; ++kh) {
            const int sg = kh < kb0 ? 0 : 1;            // segment of this block
            const int khl = sg ? kh - kb0 : kh;
            const float* p = sg ? LFI(cfptr_t, seg_ptr, 1, l) : LFI(cfptr_t, seg_ptr, 0, l);
            const int64_t ld = sg ? LFI(int64_t, seg_ld, 1, l) : LFI(int64_t, seg_ld, 0, l);
            const int k = sg ? LFI(int, seg_k, 1, l) : LFI(int, seg_k, 0, l);
            const int rd = sg ? LFI(int, seg_rd, 1, l) : LFI(int, seg_rd, 0, l);
            const int rows = sg ? LFI(int, seg_rows, 1, l) : LFI(int, seg_rows, 0, l);
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, (int)((int64_t)rows * ld * 4), RSRC_W3);
            const unsigned m = (unsigned)(st.row_ok ? sample : 0);
            const unsigned row = rd == 1 ? m : m / (unsigned)rd;
            const int col = 32 * khl + 8 * g;
            const unsigned base = (unsigned)(((int64_t)row * ld + col) * 4);
            const f4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, col < k ? base : OOB, 0, 0);
            const f4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, col + 4 < k ? base + 16 : OOB, 0, 0);
            raw[kh] = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
        }
        count_vm(c, 2 * KBH);
#pragma unroll
        for (int kh = 0; kh < KBH; ++kh) split8(raw[kh], hh[kh], hl[kh]);
    }

    f4 p = {};
    for (int nbc = 0; nbc < st.NB; ++nbc) {
        // this chunk's own DMA share has landed: every chunk issues its successor's DMA and then
        // at least EPI_MIN_VM vector-memory ops (the epilogue stores; more at layer boundaries,
        // which only makes this wait stricter), so a constant count is exact or safe
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EPI_MIN_VM) : "memory");
        barrier();               // ... and everyone else's; the other slot is free
        const int slot = c.cur;
        // this wave's 16-row block of the chunk: [kb][block][hi 1 KB | lo 1 KB]
        const char* S = c.smem + slot * SLOT_BYTES + c.half * 2048 + c.lane * 16;
        // explicit software pipeline: the fragments of k-block kb + 2 are read while kb's three
        // MFMAs run; sched_barriers pin the stages.  The previous chunk's epilogue covers the
        // latency of the first reads and fills the MFMA shadows of the first stages.
        bf16x8 fa[2], fb[2];
        auto frag = [&](int kb, bf16x8 (&f)[2]) __attribute__((always_inline)) {
            f[0] = *reinterpret_cast<const bf16x8*>(S + kb * 4096);
            f[1] = *reinterpret_cast<const bf16x8*>(S + kb * 4096 + 1024);
        };
        frag(0, fa);
        if (KB > 1) frag(1, fb);
        issue_dma(c, slot ^ 1);                        // the next chunk, a whole chunk ahead
        __builtin_amdgcn_sched_barrier(0);            // keep the DMA ahead of every other vmem op (vmcnt)
        unsigned w = 0;
        const int ep = nbc - 1;                        // the previous chunk (-1: none)
        f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            bf16x8(&f)[2] = (kb & 1) ? fb : fa;
            const bf16x8 bh = kb < KBR ? c.xh[kb < KBR ? kb : 0] : hh[kb < KBR ? 0 : kb - KBR];
            const bf16x8 bl = kb < KBR ? c.xl[kb < KBR ? kb : 0] : hl[kb < KBR ? 0 : kb - KBR];
            a = mfma_x3(f[0], f[1], bh, bl, a);
            if (kb + 2 < KB) frag(kb + 2, f);
            // the previous chunk's epilogue, one part per stage (all in the last stage if KB < 4)
            if (kb == 0) chunk_epilogue<0>(c, st, ep, p, w);
            if (kb == (KB > 1 ? 1 : 0)) chunk_epilogue<1>(c, st, ep, p, w);
            if (kb == (KB > 2 ? 2 : KB - 1)) chunk_epilogue<2>(c, st, ep, p, w);
            if (kb == (KB > 3 ? 3 : KB - 1)) chunk_epilogue<3>(c, st, ep, p, w);
            __builtin_amdgcn_sched_barrier(0);
        }
        c.cur = slot ^ 1;
        p = a;
    }
    {
        unsigned w = 0;
        const int nbc = st.NB - 1;
        chunk_epilogue<0>(c, st, nbc, p, w);
        chunk_epilogue<1>(c, st, nbc, p, w);
        chunk_epilogue<2>(c, st, nbc, p, w);
        chunk_epilogue<3>(c, st, nbc, p, w);
    }
    // the pair's halves meet: the half-1 wave hands its mask nibbles over, then both read the
    // next layer's operand image
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    if (c.half == 1) *reinterpret_cast<u2*>(c.mx + c.lane * 8) = u2{st.mw[0], st.mw[1]};
    barrier();
    if (c.half == 0) {
        const u2 o = *reinterpret_cast<const u2*>(c.mx + c.lane * 8);
        const unsigned off = st.row_ok ? (unsigned)(sample * 32 + 8 * g) : OOB;
        __builtin_amdgcn_raw_buffer_store_b64(u2{st.mw[0] | o.x, st.mw[1] | o.y}, st.rm, off, 0, 0);
        count_vm(c, 1);
    }
#pragma unroll
    for (int kb = 0; kb < KBMAX; ++kb) {
        c.xh[kb] = *reinterpret_cast<const bf16x8*>(c.xo + kb * 2048 + c.lane * 16);
        c.xl[kb] = *reinterpret_cast<const bf16x8*>(c.xo + kb * 2048 + 1024 + c.lane * 16);
    }
}

__global__ __launch_bounds__(WG, 1) void mlp_fused_fwd_kernel(FusedArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT_BYTES + NWAVE / 2 * (XO_BYTES + MX_BYTES) + BIAS_LDS];
    Ctx c;
    c.kargs = (kchar_t*)__builtin_amdgcn_kernarg_segment_ptr();
    c.smem = smem;
    c.img = a.img;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.half = c.wave & 1;
    c.xo = smem + NSLOT * SLOT_BYTES + (c.wave >> 1) * XO_BYTES;
    c.mx = smem + NSLOT * SLOT_BYTES + NWAVE / 2 * XO_BYTES + (c.wave >> 1) * MX_BYTES;
    c.bias = smem + NSLOT * SLOT_BYTES + NWAVE / 2 * (XO_BYTES + MX_BYTES);
    c.bias_base = a.bias_base;
    c.lane = threadIdx.x & 63;
    c.M = a.M;
    c.n_layers = a.n_layers;
    if ((int)blockIdx.x >= a.ntiles) return;
    const int my_tiles = (a.ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    int per_tile = 0;
    for (int l = 0; l < a.n_layers; ++l) per_tile += LF(int, nb, l);
    c.d_layer = 0;
    c.d_off = 0;
    c.d_units = LF(int, chunk_units, 0);
    c.d_left = LF(int, nb, 0);
    c.d_remaining = my_tiles * per_tile;
    c.cur = 0;
    c.after_prev = c.after_last = 0;
    // every bias of the network into LDS (offset 128: a layer's chunk -1 reads in bounds)
    for (int i = threadIdx.x * 16; i < a.bias_bytes; i += WG * 16)
        *reinterpret_cast<f4*>(const_cast<char*>(c.bias) + 128 + i) =
            *reinterpret_cast<const f4*>(a.img + a.bias_base + i);
    issue_dma(c, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the first chunk (the steady-state wait assumes successors)
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < KBMAX; ++kb) {
        c.xh[kb] = bf16x8{};
        c.xl[kb] = bf16x8{};
    }
    for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
        const int sample = tile * TILE + (c.wave >> 1) * SPW + (c.lane & 15);
        for (int l = 0; l < a.n_layers; ++l) {
            switch (LF(int, type, l)) {
                case 1: fused_layer<0, 1>(c, l, sample); break;
                case 2: fused_layer<0, 2>(c, l, sample); break;
                case 3: fused_layer<4, 0>(c, l, sample); break;
                case 6: fused_layer<8, 0>(c, l, sample); break;
                case 7: fused_layer<8, 1>(c, l, sample); break;
                case 8: fused_layer<8, 2>(c, l, sample); break;
                default: break;                          // rejected on the host
            }
        }
    }
}
#undef LF
#undef LFI

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

extern "C" int nerf_mlp_fused_fwd(const nerf_fused_layer* layers, int32_t n_layers, const void* image, int64_t M,
                                  void* stream) {
    NERF_REQUIRE(layers != nullptr && image != nullptr);
    NERF_REQUIRE(n_layers >= 1 && n_layers <= NERF_FUSED_MAX_LAYERS);
    NERF_REQUIRE(M >= 1 && M <= (int64_t)1 << 30);
    FusedArgs a;
    for (int l = 0; l < n_layers; ++l) {
        const nerf_fused_layer& L = layers[l];
        const int kbr = (L.type / 3) * 4, kbh = L.type % 3;
        NERF_REQUIRE(L.type == 1 || L.type == 2 || L.type == 3 || L.type == 6 || L.type == 7 || L.type == 8);
        NERF_REQUIRE((l == 0) == (kbr == 0));                  // only the first layer has no register input
        NERF_REQUIRE(L.N >= 1 && L.nb == (L.N + 31) / 32 && L.nb <= 16);
        NERF_REQUIRE(L.chunk_units == 4 * (kbr + kbh));
        NERF_REQUIRE(L.bias_off >= 0 && L.bias_off % 16 == 0);
        // with a second output only the first n1 chunks land in out (columns past ldo are dropped);
        // a null out (ldo 0) drops the layer's stores (inference keeps only the exposed outputs)
        NERF_REQUIRE((L.out == nullptr && L.ldo == 0) ||
                     (L.out != nullptr && aligned16(L.out) && L.ldo % 4 == 0 &&
                      L.ldo >= (L.out2 != nullptr ? (32 * L.n1 < L.N ? 32 * L.n1 : L.N) : L.N)));
        NERF_REQUIRE(M * L.ldo * 4 < ((int64_t)1 << 31));
        NERF_REQUIRE(L.mask == nullptr || (L.N <= 256 && M * 32 < ((int64_t)1 << 31)));
        NERF_REQUIRE(L.col_out == nullptr || (L.col_idx >= 0 && L.col_idx % 32 == 0 && L.col_idx < L.N));
        NERF_REQUIRE(L.img_off >= 0 && L.img_off % 1024 == 0);
        NERF_REQUIRE(L.out2 == nullptr || (aligned16(L.out2) && L.ldo2 % 4 == 0 && L.ldo2 > 0 && L.n1 >= 0 &&
                                           L.n1 <= L.nb && M * L.ldo2 * 4 < ((int64_t)1 << 31)));
        NERF_REQUIRE(L.nseg >= 0 && L.nseg <= 2);
        int kbs = 0;
        for (int s = 0; s < L.nseg; ++s) {
            NERF_REQUIRE(L.seg_ptr[s] != nullptr && aligned16(L.seg_ptr[s]));
            NERF_REQUIRE(L.seg_k[s] % 4 == 0 && L.seg_k[s] <= 32 * L.seg_kb[s] && L.seg_ld[s] % 4 == 0);
            NERF_REQUIRE(L.seg_ld[s] >= L.seg_k[s] && L.seg_rd[s] >= 1 && L.seg_rows[s] >= (M + L.seg_rd[s] - 1) / L.seg_rd[s]);
            NERF_REQUIRE((int64_t)L.seg_rows[s] * L.seg_ld[s] * 4 < ((int64_t)1 << 31));
            kbs += L.seg_kb[s];
        }
        NERF_REQUIRE(kbs == kbh);
        if (l > 0) {
            const nerf_fused_layer& P = layers[l - 1];
            const int pn = P.out2 != nullptr ? P.n1 : P.nb;
            NERF_REQUIRE(kbr <= (pn < 8 ? pn : 8));      // fed blocks exist in the previous output
        }
        a.L[l] = L;
        if (L.nseg < 2) {
            a.L[l].seg_kb[1] = 0;
            a.L[l].seg_ptr[1] = L.nseg == 1 ? L.seg_ptr[0] : nullptr;
        }
    }
    a.img = static_cast<const char*>(image);
    // the biases: contiguous, in layer order, and small enough for their LDS copy
    {
        int64_t off = layers[0].bias_off;
        for (int l = 0; l < n_layers; ++l) {
            NERF_REQUIRE(layers[l].bias_off == off);
            off += 128 * layers[l].nb;
        }
        NERF_REQUIRE(off - layers[0].bias_off + 128 <= BIAS_LDS && off < ((int64_t)1 << 31));
        a.bias_base = (int)layers[0].bias_off;
        a.bias_bytes = (int)(off - layers[0].bias_off);
    }
    a.n_layers = n_layers;
    a.M = (int)M;
    a.ntiles = (int)((M + TILE - 1) / TILE);
    const int grid = a.ntiles < num_cus() ? a.ntiles : num_cus();
    hipLaunchKernelGGL(mlp_fused_fwd_kernel, dim3(grid), dim3(WG), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
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
