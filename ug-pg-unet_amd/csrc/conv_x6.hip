// 3x3 / pad-1 convolution forward and data-gradient on bf16 MFMA with fp32
// accuracy ("split-bf16 x6"), gfx950.
//
// Every fp32 operand x is split exactly into three bf16 pieces
//     x = x0 + x1 + x2,  x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)
// (round-to-nearest; each remainder is exact in fp32, and 3 x 8 significand bits
// cover fp32's 24).  A product keeps the six terms of order <= 2,
//     a*b ~ a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0,
// dropping a1 b2 + a2 b1 + a2 b2, which is below 2^-25 |a b| -- under the
// rounding error of one fp32 multiply.  bf16 x bf16 products are exact in the
// fp32 accumulator, so each output is an fp32 sum of fp32-accurate products:
// the same arithmetic class as the v_mfma_f32_32x32x2_f32 path in conv.hip, at
// 6 x v_mfma_f32_32x32x16_bf16 (6 x 32 cycles) per 16-deep k-step instead of
// 8 x v_mfma_f32_32x32x2_f32 (8 x 64 cycles): 2.67x the MFMA rate.
//
// Tile: 128 output pixels (4 x 32, or 8 x 16 for narrow images) x 64 output
// channels, input channels in chunks of 16 (one MFMA k-step per tap).  The
// activation halo is staged in LDS as three bf16 planes, split while staging
// (after the lazy BatchNorm+ReLU of the producer); the weights arrive pre-split
// by launch_pack_x6 in exactly the LDS image order.  4 waves as 2 (pixels) x 2
// (channels), each a 64 x 32 output block = two 32x32 accumulators.
//
// LDS images (16-byte vectors of 8 bf16):
//   A [piece 3][channel half 2][NHP]  pixel pitch 16 B, halo row pitch HS
//   B [piece 3][channel half 2][tap 9][co 64]
// Both fragment reads are single ds_read_b128 per (piece, tile) and conflict-free:
// a 16-lane read group touches 16 distinct 16-B bank slots (32-wide tile: one
// image row; 16-wide tile: permuted rows, see tile_pixel<16, true>, with HS=24).
#include <algorithm>
#include <atomic>
#include <type_traits>

#include "conv_common.h"

namespace ugpg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// (a, b) rounded to bf16 (nearest even) and packed, a in the low half (one
// v_cvt_pk_bf16_f32); the two rounded values are recovered from the packed word by
// bit operations, so no element is converted twice
__device__ __forceinline__ unsigned pk_bf16(float a, float b, float& ra, float& rb) {
    const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
    ra = __builtin_bit_cast(float, u << 16);
    rb = __builtin_bit_cast(float, u & 0xffff0000u);
    return u;
}
// the three bf16 pieces of a pair: x = hi + mid + lo to fp32 accuracy
__device__ __forceinline__ void split3_pair(float a, float b, unsigned& u0, unsigned& u1,
                                            unsigned& u2) {
    float ha, hb;
    u0 = pk_bf16(a, b, ha, hb);
    a -= ha;
    b -= hb;
    u1 = pk_bf16(a, b, ha, hb);
    a -= ha;
    b -= hb;
    u2 = pk_bf16(a, b, ha, hb);
}

__device__ __forceinline__ void split3(f32x8 v, u32x4& p0, u32x4& p1, u32x4& p2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        unsigned a, b, c;
        split3_pair(v[2 * i], v[2 * i + 1], a, b, c);
        p0[i] = a;
        p1[i] = b;
        p2[i] = c;
    }
}

// compute units of the stream's device (cached per device; relaxed atomics: entries are
// written once with the same value, from any host thread)
static int cu_count(hipStream_t st) {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    }
    int n = cache[dev].load(std::memory_order_relaxed);
    if (!n) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0)
            n = 256;
        cache[dev].store(n, std::memory_order_relaxed);
    }
    return n;
}

// identity lazy-activation coefficients (for sources stored already activated)
__device__ const float g_act_ones[1024] = {
#define UGPG_ONE8 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f
#define UGPG_ONE64 UGPG_ONE8, UGPG_ONE8, UGPG_ONE8, UGPG_ONE8, UGPG_ONE8, UGPG_ONE8, UGPG_ONE8, UGPG_ONE8
    UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64,
    UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64, UGPG_ONE64};
#undef UGPG_ONE64
#undef UGPG_ONE8
__device__ const float g_act_zeros[1024] = {0.f};

// max(scale*v + shift, floor): the lazy BatchNorm+ReLU with floor 0, the identity
// with scale 1, shift 0, floor -inf (no branch on whether the source has one)
__device__ __forceinline__ f32x4 act_floor4(f32x4 v, const Act4& a, float lo) {
    v.x = fmaxf(fmaf(v.x, a.s.x, a.h.x), lo);
    v.y = fmaxf(fmaf(v.y, a.s.y, a.h.y), lo);
    v.z = fmaxf(fmaf(v.z, a.s.z, a.h.z), lo);
    v.w = fmaxf(fmaf(v.w, a.s.w, a.h.w), lo);
    return v;
}

__device__ __forceinline__ f32x16 mfma16(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 mfma16x16(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// sum over the 16 lanes of a DPP row, result in every lane of the row
__device__ __forceinline__ float row16_sum(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0xB1, 0xF, 0xF, false));  // [1,0,3,2]
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0x4E, 0xF, 0xF, false));  // [2,3,0,1]
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0x141, 0xF, 0xF, false));  // half mirror
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0x140, 0xF, 0xF, false));  // mirror
    return v;
}

// acc += a*b from the pieces: NP = 3 -> fp32 accuracy (the six products of order
// <= 2, smallest terms first); NP = 1 -> one bf16 product (the "bf16" arithmetic of
// BASELINE config 3: operands rounded to bf16, fp32 accumulation)
template <int NP>
__device__ __forceinline__ f32x16 mfma_xn(const u32x4 (&a)[NP], const u32x4 (&b)[NP], f32x16 c) {
    if constexpr (NP == 3) {
        c = mfma16(a[2], b[0], c);
        c = mfma16(a[1], b[1], c);
        c = mfma16(a[0], b[2], c);
        c = mfma16(a[1], b[0], c);
        c = mfma16(a[0], b[1], c);
    }
    c = mfma16(a[0], b[0], c);
    return c;
}
__device__ __forceinline__ f32x16 mfma_x6(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16 c) {
    return mfma_xn<3>(a, b, c);
}
// the first NP pieces of x (NP = 1: bf16(x), round to nearest even)
template <int NP>
__device__ __forceinline__ void split_n(f32x8 v, u32x4 (&p)[NP]) {
    if constexpr (NP == 3) {
        split3(v, p[0], p[1], p[2]);
    } else {
        p[0] = __builtin_bit_cast(u32x4, __builtin_convertvector(v, bf16x8));
    }
}

template <int TH, int TW, bool PERM16, int NP>
__global__ void __launch_bounds__(256) conv3x3_fwd_x6_kernel(ConvFwdArgs a) {
    constexpr int BN = 64, BKC = 16, WM = 2, WN = 2, MT = 2, NT = 1;
    static_assert(TH * TW == 128, "tile must be 128 pixels");
    constexpr int HWD = TW + 2;                  // halo width
    constexpr int HS = PERM16 ? 24 : HWD;        // halo row pitch in the LDS image
    constexpr int NHALO = (TH + 2) * HWD;        // staged halo pixels
    constexpr int NHP0 = (TH + 2) * HS;
    constexpr int NHP = NHP0 + (12 - NHP0 % 8) % 8;  // = 4 (mod 8): h planes 64 B apart mod 128
    constexpr int A_ITEMS = NHALO * 2;           // (pixel, channel half) items
    constexpr int A_PER = (A_ITEMS + 255) / 256;
    constexpr int B_VEC = 2 * NP * 9 * BN;       // 16-B vectors of the weight slab
    constexpr int B_PER = (B_VEC + 255) / 256;
    constexpr int A_VECS = 2 * NP * NHP;
    __shared__ __attribute__((aligned(16))) u32x4 smem[A_VECS + B_VEC];
    u32x4* As = smem;
    u32x4* Bs = smem + A_VECS;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int NB = a.Cout / BN;
    const int nb = blockIdx.x % NB, tile = blockIdx.x / NB;
    const int n0 = nb * BN;
    const int tpi = a.tiles_x * a.tiles_y;
    const int b = tile / tpi, trem = tile % tpi;
    const int ty0 = (trem / a.tiles_x) * TH, tx0 = (trem % a.tiles_x) * TW;
    const int nchunk = a.Cin / BKC;

    f32x4 ra[A_PER][2];
    u32x4 rb[B_PER];
    unsigned avalid = 0;
    Act4 ract0, ract1;
    bool aon = false;

    auto gload = [&](int c) {
        int cb = c * BKC;
        const float* src = a.src0;
        const float* sc = a.sc0;
        const float* sh = a.sh0;
        int Cs = a.C0;
        if (cb >= a.C0) {
            src = a.src1;
            sc = a.sc1;
            sh = a.sh1;
            Cs = a.C1;
            cb -= a.C0;
        }
        // this thread's channel half is fixed (hh = idx & 1 = tid & 1); an 8-channel
        // source is zero-extended to the 16-channel chunk (upper half never read)
        const bool cok = cb + (tid & 1) * 8 < Cs;
        const int ch = cb + (cok ? (tid & 1) * 8 : 0);
        aon = sc != nullptr;
        ract0 = act_load4(sc, sh, ch);
        ract1 = act_load4(sc, sh, ch + 4);
        avalid = 0;
        // branch-free: every lane loads from a clamped (valid) address and the halo
        // mask is applied at LDS-store time, so no loaded register is merged at a
        // join (which makes the compiler wait for the prefetch before the MFMAs)
#pragma unroll
        for (int v = 0; v < A_PER; ++v) {
            const int idx = tid + v * 256;
            const int hp = idx < A_ITEMS ? idx >> 1 : 0;
            const int gy = ty0 - 1 + hp / HWD, gx = tx0 - 1 + hp % HWD;
            const bool ok = cok && idx < A_ITEMS && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W;
            const int cy = min(max(gy, 0), a.H - 1), cx = min(max(gx, 0), a.W - 1);
            const float* p = src + ((size_t)(b * a.H + cy) * a.W + cx) * Cs + ch;
            ra[v][0] = *reinterpret_cast<const f32x4*>(p);
            ra[v][1] = *reinterpret_cast<const f32x4*>(p + 4);
            avalid |= (ok ? 1u : 0u) << v;
        }
        const u32x4* wsrc = static_cast<const u32x4*>(a.wpk) + ((size_t)nb * nchunk + c) * B_VEC;
#pragma unroll
        for (int v = 0; v < B_PER; ++v) rb[v] = wsrc[min(tid + v * 256, B_VEC - 1)];
    };

    auto lstore = [&](int c) {
        (void)c;
#pragma unroll
        for (int v = 0; v < A_PER; ++v) {
            const int idx = tid + v * 256;
            if (idx < A_ITEMS) {
                const int hp = idx >> 1, hh = idx & 1;
                f32x4 lo4 = act_reg4(ra[v][0], ract0, aon), hi4 = act_reg4(ra[v][1], ract1, aon);
                if (!((avalid >> v) & 1u)) lo4 = hi4 = f32x4{0.f, 0.f, 0.f, 0.f};
                const f32x8 x = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
                u32x4 pc[NP];
                split_n<NP>(x, pc);
                const int hl = (hp / HWD) * HS + hp % HWD;
#pragma unroll
                for (int q = 0; q < NP; ++q) As[(q * 2 + hh) * NHP + hl] = pc[q];
            }
        }
#pragma unroll
        for (int v = 0; v < B_PER; ++v) {
            const int idx = tid + v * 256;
            if (idx < B_VEC) Bs[idx] = rb[v];
        }
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mt][0][r] = 0.f;

    const int hl = lane >> 5;
    int aoff[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = tile_pixel<TW, PERM16>(wm * 64 + mt * 32 + (lane & 31));
        aoff[mt] = hl * NHP + (m / TW) * HS + (m % TW);
    }
    const int boff = hl * 3 * BN + wn * 32 + (lane & 31);

    auto ldfrag = [&](int t, u32x4 (&af)[MT][NP], u32x4 (&bf)[NP]) {
        const int toff = (t / 3) * HS + (t % 3);
#pragma unroll
        for (int q = 0; q < NP; ++q) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) af[mt][q] = As[q * 2 * NHP + aoff[mt] + toff];
            bf[q] = Bs[(((t / 3) * NP + q) * 2) * 3 * BN + boff + (t % 3) * BN];
        }
    };

    gload(0);
    lstore(0);
    __syncthreads();
    for (int c = 0; c < nchunk; ++c) {
        if (c + 1 < nchunk) gload(c + 1);
        u32x4 fa[2][MT][NP], fb[2][NP];
        ldfrag(0, fa[0], fb[0]);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            if (t + 1 < 9) ldfrag(t + 1, fa[(t + 1) & 1], fb[(t + 1) & 1]);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[mt][0] = mfma_xn<NP>(fa[t & 1][mt], fb[t & 1], acc[mt][0]);
        }
        __syncthreads();
        if (c + 1 < nchunk) {
            lstore(c + 1);
            __syncthreads();
        }
    }

    conv_epilogue<TH, TW, BN, WM, WN, MT, NT, PERM16>(a, acc, reinterpret_cast<float*>(smem), tile,
                                                      b, ty0, tx0, n0, wm, wn);
}

// ---------------------------------------------------------------------------
// Persistent, warp-specialized form of the same forward for images >= 32 wide
// ("x6r").  One 8-wave workgroup per CU; a work item is an 8 x 32 = 256-pixel tile
// x 64 output channels (twice the pixels of conv3x3_fwd_x6_kernel, so each weight
// byte staged through the CU feeds twice the MFMAs -- the per-CU L2->LDS weight
// stream is what bounds the single-stage kernel).  Waves 0-3 only read fragments
// and issue MFMAs (2 pixel halves x 2 column halves, each 128 px x 32 co = four
// 32x32 accumulators); waves 4-7 only stage.  The K loop runs per 16-channel
// chunk ("step") in three phases, one per kernel row ky: the halo is double-
// buffered per step (2 x 33 KB) and the weights go through a ring of four
// kernel-row slots (4 x 18 KB), so the loaders write row r of step k+1 while
// row r of step k is being computed, with one barrier per phase.  Items are
// walked per XCD as contiguous ranges (column blocks of one tile share the halo
// in one L2).  Epilogue per wave, no barriers: BatchNorm partials per (tile,
// pixel half), i.e. 2 stat slots per tile.
// ---------------------------------------------------------------------------
// 16-byte global load the compiler does not track: the caller waits for it with an
// explicit counted s_waitcnt vmcnt (vm_wait), which is followed by a scheduling
// fence.  The loader waves use it so that their loads stay in flight across
// barriers and loop iterations (hipcc's own waitcnt placement drains all loads at
// loop headers).
__device__ __forceinline__ f32x4 gld16(const void* p) {
    f32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p));
    return r;
}
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
// the same for 8 bytes (4 bf16)
__device__ __forceinline__ u32x2v gld8(const void* p) {
    u32x2v r;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(p));
    return r;
}
// ... and 4 bytes
__device__ __forceinline__ unsigned gld4(const void* p) {
    unsigned r;
    asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p));
    return r;
}
// LDS-DMA: 16 bytes per lane from g (per-lane address) to lds_wave + 16*lane (lds_wave
// wave-uniform), counted by vmcnt like a load; no VGPR destination
__device__ __forceinline__ void glds16(const void* g, void* lds_wave) {
    const unsigned m0 =
        __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<uintptr_t>(lds_wave));
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g), "s"(m0)
        : "memory");
}
// N (<= 4) consecutive 1-KiB LDS-DMA blocks of one wave: global g + 1024 i -> LDS
// lds_wave + 1024 i + 16 lane.  The instruction offset applies to both addresses, so M0 is
// set once per run (the per-block M0 switches -- readfirstlane, s_mov, s_nop, restore --
// were the bulk of the loaders' DMA issue)
template <int N>
__device__ __forceinline__ void glds16_run(const void* g, void* lds_wave) {
    static_assert(N >= 1 && N <= 4, "13-bit instruction offsets: at most 4 blocks per run");
    const unsigned m0 =
        __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<uintptr_t>(lds_wave));
    unsigned keep;
    if constexpr (N == 1)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(m0) : "memory");
    else if constexpr (N == 2)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, off\n\t"
                     "global_load_lds_dwordx4 %1, off offset:1024\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(m0) : "memory");
    else if constexpr (N == 3)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, off\n\t"
                     "global_load_lds_dwordx4 %1, off offset:1024\n\t"
                     "global_load_lds_dwordx4 %1, off offset:2048\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(m0) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, off\n\t"
                     "global_load_lds_dwordx4 %1, off offset:1024\n\t"
                     "global_load_lds_dwordx4 %1, off offset:2048\n\t"
                     "global_load_lds_dwordx4 %1, off offset:3072\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(m0) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
    __builtin_amdgcn_sched_barrier(0);
}
// workgroup barrier for waves that write no LDS: their fragment reads for the next
// phase (a different ring slot than the one the loaders overwrite next) stay in flight
__device__ __forceinline__ void read_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
// LDS writes complete, then a workgroup barrier that does not wait for global loads
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// per-wave epilogue: bias, (dual-destination, accumulate-capable) store, and the
// wave's BatchNorm partial (count, sum, M2) over its MT*32 pixels x 32 channels into
// slot 2*tile + wm (stat slots = 2 * ntiles).  Each 32-pixel MFMA tile is one image
// row (TW == 32): lane (h, c) holds pixels (r&3) + 8(r>>2) + 4h of row wm*MT + mt,
// channel c, so addresses are one row base + a per-lane offset + a constant per r;
// the accumulate and bounds decisions are uniform per item.
//
// bf16-only storage (the forward under bf16 arithmetic): the lane layout above holds one
// channel of 16 pixels, so direct stores are 2 bytes per lane (64-byte segments, 16
// store instructions per m-tile -- measured: half of the K = 64 layers' loop time in
// the epilogue).  Instead each m-tile goes through the wave's LDS staging area `stg`
// (32 pixels x 40 floats: the two pixel halves h land on opposite bank halves) and
// leaves as 16-byte stores of 8 channels (2 per lane per m-tile).
#ifdef X6R_STAMP
// diagnostic build: cycles of the last epilogue of each workgroup's first compute wave in
// its store phase and its statistics phase
__device__ unsigned long long g_epi[512 * 4];
#define EPI_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define EPI_REC(t0, t1)                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 512) {                               \
        g_epi[4 * blockIdx.x] = t1 - t0;                                      \
        g_epi[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memtime() - t1;        \
    }
#else
#define EPI_T(v)
#define EPI_REC(t0, t1)
#endif
#ifndef X6R_PAIR16  // (A/B build: X6R_PAIR16=0, each n-tile through x6_epilogue_wave)
#define X6R_PAIR16 1
#endif
#ifndef X6R_PAIR16_BNB  // (A/B build: X6R_PAIR16_BNB=0, data gradients with partials per n-tile)
#define X6R_PAIR16_BNB 1
#endif
constexpr int X6_STG_PITCH = 40;
constexpr int X6_STG_WAVE = 2048;  // floats: 32 x 40 fp32, or the bf16 y tile of 4 m-tiles
// BatchNorm-backward partials with bf16 y: the item's y tile (MT m-tiles x 32 pixels x the
// wave's 32 channels) DMA'd into the wave's staging area as [mt][pixel][channel] bf16
// (2 KiB per m-tile; 16 bytes per lane: pixel (lane>>2) + 16j, channels 8(lane&3)..)
template <int TH, int TW, int MT>
__device__ __forceinline__ void x6_dma_bnb_y(const ConvFwdArgs& a, int b, int ty0, int tx0, int c0,
                                             int wm, float* stg) {
    const int lane = threadIdx.x & 63;
    const int vh = min(TH, a.H - ty0), vw = min(TW, a.W - tx0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int py = min(wm * MT + mt, vh - 1);  // rows past the image: never read back
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int px = min((lane >> 2) + 16 * j, vw - 1), k = lane & 3;
            const __bf16* g = a.bnb_y.h + ((size_t)(b * a.H + ty0 + py) * a.W + tx0 + px) * a.Cout +
                              c0 + 8 * k;
            glds16(g, reinterpret_cast<char*>(stg) + (mt * 2 + j) * 1024);
        }
    }
}
// Y32: the BatchNorm-backward partials may read an fp32 y (the 4 x 2-tile single-piece
// forms need a bf16 y -- the host routes the rest to the 4 x 1 form -- which keeps this
// path, and its registers, out of them).  FW: the tile is known to lie wholly inside the
// image width (the caller's uniform branch), so no store or statistics term carries a
// per-pixel column guard (each was an exec-mask branch per value)
template <int TH, int TW, int MT, int WM = 2, bool Y32 = true, bool FW = false>
__device__ __forceinline__ void x6_epilogue_wave(const ConvFwdArgs& a, f32x16 (&acc)[MT], int tile,
                                                 int b, int ty0, int tx0, int c0, int wm,
                                                 float* stg) {
    static_assert(TW == 32, "one image row per 32-pixel MFMA tile");
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int vh = min(TH, a.H - ty0), vw = min(TW, a.W - tx0);
    const bool fullw = FW || vw == TW;
    float* out;
    int ostride, ocol0, oacc;
    if (c0 < a.split) {  // (a 32-wide n-tile never straddles the split: split % 64 == 0)
        out = a.out0;
        ostride = a.split;
        ocol0 = c0;
        oacc = a.acc0;
    } else {
        out = a.out1;
        ostride = a.Cout - a.split;
        ocol0 = c0 - a.split;
        oacc = a.acc1;
    }
    const int l32 = lane & 31;
    const float bv = a.bias ? a.bias[c0 + l32] : 0.f;
    const int lane_off = 4 * h * ostride + ocol0 + l32;
    // bf16 storage only (out0 == nullptr, one output): the stored -- rounded -- values are
    // the ones the BatchNorm statistics describe
    const bool only16 = out == nullptr;
    float psum = 0.f;
    // the stores of m-tiles [m0, m1)
    auto store_rows = [&](auto accumulate, int m0, int m1) {
        constexpr bool ACC = decltype(accumulate)::value;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            if (mt < m0 || mt >= m1) continue;
            const int py = wm * MT + mt;
            if (py >= vh) break;  // uniform
            const size_t rowe = (size_t)((b * a.H + ty0 + py) * a.W + tx0) * ostride + lane_off;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int pxc = (r & 3) + 8 * (r >> 2);  // + 4h in lane_off
                float v = acc[mt][r] + bv;
                if (!ACC && only16) v = (float)(__bf16)v;
                acc[mt][r] = v;
                if (fullw || pxc + 4 * h < vw) {
                    const size_t e = rowe + (size_t)pxc * ostride;
                    if constexpr (ACC) {
                        out[e] += v;
                    } else {
                        if (!only16) out[e] = v;
                        if (a.out0_16)  // bf16 storage or copy (one output: ostride == Cout)
                            a.out0_16[e] = (__bf16)v;
                    }
                    psum += v;
                }
            }
            // one m-tile's loads in flight at a time (the accumulate path's 64 loads at once
            // cost the 4 x 2-tile forms their register headroom)
            asm volatile("" ::: "memory");
        }
    };
    // bf16-only storage through the staging area (no accumulate).  FINAL: acc already holds
    // the rounded values with bias (the data gradient's epilogue with BatchNorm-backward
    // partials rounds before its partials), else bias, rounding and the statistics sum here
    auto store16_rows = [&](auto final_) {
        constexpr bool FINAL = decltype(final_)::value;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int py = wm * MT + mt;
            if (py >= vh) break;  // uniform
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                float v0 = acc[mt][r], v1 = acc[mt][r + 1];
                if constexpr (!FINAL) {
                    pk_bf16(v0 + bv, v1 + bv, v0, v1);
                    acc[mt][r] = v0;
                    acc[mt][r + 1] = v1;
                }
                const int p0 = (r & 3) + 8 * (r >> 2) + 4 * h;  // r + 1: pixel p0 + 1
                if constexpr (!FINAL) {
                    if (fullw || p0 < vw) psum += v0;
                    if (fullw || p0 + 1 < vw) psum += v1;
                }
                stg[p0 * X6_STG_PITCH + l32] = v0;
                stg[(p0 + 1) * X6_STG_PITCH + l32] = v1;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const size_t rowb = (size_t)((b * a.H + ty0 + py) * a.W + tx0) * ostride + ocol0;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int p = (lane >> 2) + 16 * j, k = lane & 3;
                const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + p * X6_STG_PITCH + 8 * k);
                const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + p * X6_STG_PITCH + 8 * k + 4);
                // exact bf16 values: the packed words are bit selections
                auto pk = [](float x, float y) {
                    return (__builtin_bit_cast(unsigned, x) >> 16) |
                           (__builtin_bit_cast(unsigned, y) & 0xffff0000u);
                };
                const u32x4 w = {pk(lo.x, lo.y), pk(lo.z, lo.w), pk(hi.x, hi.y), pk(hi.z, hi.w)};
#ifdef X6Q_NOSTORE  // diagnostic build: no output stores (results are wrong)
                if (w[0] == 0x12345678u)
#else
                if (fullw || p < vw)
#endif
#ifndef X6_PLAIN_STORES  // (A/B build: plain stores)
                    // non-temporal bf16 output stores: forward launches 3-5 % faster, bf16 step
                    // -0.6 % in-process (profiles/r6f_ab_nontemporal_epilogue_stores.txt)
                    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(a.out0_16 + rowb + (size_t)p * ostride + 8 * k));
#else
                    *reinterpret_cast<u32x4*>(a.out0_16 + rowb + (size_t)p * ostride + 8 * k) = w;
#endif
            }
            asm volatile("" ::: "memory");  // the next m-tile's staging writes after these reads
        }
    };
    const bool bnb = a.bnb_part != nullptr && !oacc;  // (the host refuses bnb + accumulate)
    EPI_T(et0);
    if (oacc) store_rows(std::integral_constant<bool, true>{}, 0, MT);
    else if (only16 && !bnb) store16_rows(std::false_type{});
    else if (!bnb) store_rows(std::integral_constant<bool, false>{}, 0, MT);
    EPI_T(et1);
    if (bnb) {
        // BatchNorm-backward partials of the stored output (as x6q_epilogue_wave): this
        // lane's channel over its pixels, the two pixel halves (h) combined by a shuffle
        const int n = c0 + l32;
        const float mu = a.bnb_mean[n], is = a.bnb_invstd[n], sc = a.bnb_scale[n],
                    sh = a.bnb_shift[n];
        float sg = 0.f, sgx = 0.f, sx = 0.f;
        if (a.bnb_y.h) vm_wait<0>();  // the staged y tile has landed
        auto part = [&](int mt, int r, float y) {
            const int pxc = (r & 3) + 8 * (r >> 2);
            if (fullw || pxc + 4 * h < vw) {
                const float gv = fmaf(y, sc, sh) > 0.f ? acc[mt][r] : 0.f;
                const float xh = (y - mu) * is;
                sg += gv;
                sgx = fmaf(gv, xh, sgx);
                sx += xh;
            }
        };
        if (a.bnb_y.h) {
            // bf16 y: the item's tile was DMA'd into the staging area during its last step
            // (conv3x3_fwd_x6r_kernel, x6_dma_bnb_y); lane (h, c) reads channel c of its
            // pixels (2-byte gathers from HBM ran the data gradient at half the forward's
            // speed).  The partials of every m-tile first, then the fp32 output leaves
            // through the same staging area as 16-byte stores of 4 channels (4 per lane and
            // m-tile instead of 16 4-byte ones; pitch 32 floats: conflict-free both ways)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                if (wm * MT + mt >= vh) break;  // uniform
                const __bf16* t16 = reinterpret_cast<const __bf16*>(stg) + mt * 1024 + (lane & 31);
#pragma unroll
                for (int r = 0; r < 16; r += 2) {
                    // bf16-only output (the bf16 arithmetic's data gradient): the partials
                    // describe the stored, rounded values
                    float v0 = acc[mt][r] + bv, v1 = acc[mt][r + 1] + bv;
                    if (only16) pk_bf16(v0, v1, v0, v1);
                    acc[mt][r] = v0;
                    acc[mt][r + 1] = v1;
                    part(mt, r, (float)t16[((r & 3) + 8 * (r >> 2) + 4 * h) * 32]);
                    part(mt, r + 1, (float)t16[(((r + 1) & 3) + 8 * ((r + 1) >> 2) + 4 * h) * 32]);
                }
                asm volatile("" ::: "memory");  // (as store_rows: one m-tile's reads at a time)
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // y reads done: reuse the area
            if (only16) store16_rows(std::true_type{});
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                if (only16) break;  // (stored above)
                const int py = wm * MT + mt;
                if (py >= vh) break;  // uniform
#pragma unroll
                for (int r = 0; r < 16; ++r) stg[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + l32] = acc[mt][r];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const size_t rowb = (size_t)((b * a.H + ty0 + py) * a.W + tx0) * ostride + ocol0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int p = (lane >> 3) + 8 * j, k = lane & 7;
                    const f32x4 v = *reinterpret_cast<const f32x4*>(stg + p * 32 + 4 * k);
                    if (fullw || p < vw) *reinterpret_cast<f32x4*>(out + rowb + (size_t)p * ostride + 4 * k) = v;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads before the next m-tile's writes
            }
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int py = wm * MT + mt;
            if (py >= vh) break;  // uniform
            if (!Y32 || a.bnb_y.h) {
                break;  // (done above)
            } else {
                float yv[16];
                const size_t yrow = (size_t)((b * a.H + ty0 + py) * a.W + tx0 + 4 * h) * a.Cout + n;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int pxc = min((r & 3) + 8 * (r >> 2), vw - 1 - 4 * h);
                    yv[r] = a.bnb_y.f[yrow + (size_t)max(pxc, -4 * h) * a.Cout];
                }
                // this row's output stores issue while its y loads are in flight
                store_rows(std::integral_constant<bool, false>{}, mt, mt + 1);
#pragma unroll
                for (int r = 0; r < 16; ++r) part(mt, r, yv[r]);
            }
        }
        sg += __shfl_xor(sg, 32, 64);
        sgx += __shfl_xor(sgx, 32, 64);
        sx += __shfl_xor(sx, 32, 64);
        if (lane < 32) {
            const size_t S = WM * (size_t)a.ntiles, slot = WM * (size_t)tile + wm;
            a.bnb_part[(0 * (size_t)a.Cout + n) * S + slot] = sg;
            a.bnb_part[(1 * (size_t)a.Cout + n) * S + slot] = sgx;
            a.bnb_part[(2 * (size_t)a.Cout + n) * S + slot] = sx;
        }
        return;
    }
    if (a.stats == nullptr) return;
#ifdef X6Q_NOSTATS
    return;
#endif
    constexpr int WROWS = MT * 32 / TW;  // image rows of one wave's pixels
    const int rows = min(max(vh - wm * WROWS, 0), WROWS);
    const float cnt = (float)(rows * vw);
    const float s = psum + __shfl_xor(psum, 32, 64);
    const float mu = cnt > 0.f ? s / cnt : 0.f;
    float q = 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        if (wm * MT + mt >= vh) break;  // uniform
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int px = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (fullw || px < vw) {
                const float d = acc[mt][r] - mu;
                q = fmaf(d, d, q);
            }
        }
    }
    q += __shfl_xor(q, 32, 64);
    if (lane < 32) {
        const size_t n = c0 + l32, S = WM * (size_t)a.ntiles, slot = WM * (size_t)tile + wm;
        a.stats[(0 * (size_t)a.Cout + n) * S + slot] = cnt;
        a.stats[(1 * (size_t)a.Cout + n) * S + slot] = s;
        a.stats[(2 * (size_t)a.Cout + n) * S + slot] = q;
    }
    EPI_REC(et0, et1);
}

// The 4 x 2-tile single-piece forms' common epilogue -- bf16-only output, no accumulate, no
// BatchNorm-backward partials, a full-width tile: the wave's two n-tiles are one pixel's 64
// channels, i.e. one whole 128-B line of the bf16 output, so each m-tile leaves as 4 store
// instructions of 8 lanes x 16 B per line (x6_epilogue_wave per n-tile writes half lines:
// a CU retires those at ~31 GB/s against ~78 GB/s for whole lines, tools/store_probe.cpp).
// Staging pitch 32 floats and the second n-tile's area 4 dwords off: conflict-free for the
// stores (ds_write_b32) and for the line reads (ds_read_b128 lane groups).  The
// BatchNorm partials are taken in one pass as shifted sums (K = a value of the channel,
// d = v - K: sum = n K + sum d, M2 = sum d^2 - (sum d)^2 / n), so each m-tile's
// accumulators die once staged; the two-pass form held all of them to its second pass (the
// round-6 paired store that rounded both tiles first spilled 480 B).
template <int TH, int TW, int MT, int WM>
__device__ __forceinline__ void x6_epilogue_pair16(const ConvFwdArgs& a, f32x16 (&acc0)[MT],
                                                   f32x16 (&acc1)[MT], int tile, int b, int ty0,
                                                   int tx0, int c0, int wm, float* stg) {
    static_assert(TW == 32, "one image row per 32-pixel MFMA tile");
    constexpr int P = 32;
    const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const int vh = min(TH, a.H - ty0);
    float* const stg1 = stg + X6_STG_WAVE + 4;
    const float bv0 = a.bias ? a.bias[c0 + l32] : 0.f, bv1 = a.bias ? a.bias[c0 + 32 + l32] : 0.f;
    // the shift of channel c0 + l32 (+ 32): lane l32's first value, the same in both halves
    const float k0 = __shfl(acc0[0][0] + bv0, l32, 64), k1 = __shfl(acc1[0][0] + bv1, l32, 64);
    float s0 = 0.f, q0 = 0.f, s1 = 0.f, q1 = 0.f;
    auto pk = [](float x, float y) {  // exact bf16 values: the packed words are bit selections
        return (__builtin_bit_cast(unsigned, x) >> 16) | (__builtin_bit_cast(unsigned, y) & 0xffff0000u);
    };
    const int k = lane & 7;
    const float* const sk = (k < 4 ? stg : stg1) + 8 * (k & 3);
    EPI_T(et0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int py = wm * MT + mt;
        if (py >= vh) break;  // uniform
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const int p0 = (r & 3) + 8 * (r >> 2) + 4 * h;  // r + 1: pixel p0 + 1
            float v0, v1, w0, w1;
            pk_bf16(acc0[mt][r] + bv0, acc0[mt][r + 1] + bv0, v0, v1);
            pk_bf16(acc1[mt][r] + bv1, acc1[mt][r + 1] + bv1, w0, w1);
            float d = v0 - k0;
            s0 += d;
            q0 = fmaf(d, d, q0);
            d = v1 - k0;
            s0 += d;
            q0 = fmaf(d, d, q0);
            d = w0 - k1;
            s1 += d;
            q1 = fmaf(d, d, q1);
            d = w1 - k1;
            s1 += d;
            q1 = fmaf(d, d, q1);
            stg[p0 * P + l32] = v0;
            stg[(p0 + 1) * P + l32] = v1;
            stg1[p0 * P + l32] = w0;
            stg1[(p0 + 1) * P + l32] = w1;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const size_t rowb = (size_t)((b * a.H + ty0 + py) * a.W + tx0) * a.Cout + c0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int p = (lane >> 3) + 8 * j;
            const f32x4 lo = *reinterpret_cast<const f32x4*>(sk + p * P);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(sk + p * P + 4);
            const u32x4 w = {pk(lo.x, lo.y), pk(lo.z, lo.w), pk(hi.x, hi.y), pk(hi.z, hi.w)};
            __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(a.out0_16 + rowb + (size_t)p * a.Cout + 8 * k));
        }
        asm volatile("" ::: "memory");  // the next m-tile's staging writes after these reads
    }
    EPI_T(et1);
    s0 += __shfl_xor(s0, 32, 64);
    q0 += __shfl_xor(q0, 32, 64);
    s1 += __shfl_xor(s1, 32, 64);
    q1 += __shfl_xor(q1, 32, 64);
    if (a.stats != nullptr && lane < 32) {
        const int rows = min(max(vh - wm * MT, 0), MT);
        const float cnt = (float)(rows * TW);
        const size_t S = WM * (size_t)a.ntiles, slot = WM * (size_t)tile + wm;
        auto put = [&](int n, float kk, float s, float q) {
            const bool any = cnt > 0.f;
            a.stats[(0 * (size_t)a.Cout + n) * S + slot] = cnt;
            a.stats[(1 * (size_t)a.Cout + n) * S + slot] = any ? fmaf(cnt, kk, s) : 0.f;
            a.stats[(2 * (size_t)a.Cout + n) * S + slot] = any ? fmaxf(q - s * (s / cnt), 0.f) : 0.f;
        };
        put(c0 + l32, k0, s0, q0);
        put(c0 + 32 + l32, k1, s1, q1);
    }
    EPI_REC(et0, et1);
}

// The same forms' data-gradient epilogue with BatchNorm-backward partials (bf16-only da, bf16
// y, no accumulate, full-width tile): pass 1 rounds both n-tiles and takes their partials
// from the y tiles DMA'd into the two staging areas (x6_dma_bnb_y; each n-tile's values,
// order and rounding exactly as x6_epilogue_wave's bnb path), pass 2 sends each m-tile out as
// whole 128-B lines through the then free staging (as x6_epilogue_pair16)
template <int TH, int TW, int MT, int WM>
__device__ __forceinline__ void x6_epilogue_pair16_bnb(const ConvFwdArgs& a, f32x16 (&acc0)[MT],
                                                       f32x16 (&acc1)[MT], int tile, int b, int ty0,
                                                       int tx0, int c0, int wm, float* stg) {
    static_assert(TW == 32, "one image row per 32-pixel MFMA tile");
    constexpr int P = 32;
    const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const int vh = min(TH, a.H - ty0);
    float* const stg1 = stg + X6_STG_WAVE + 4;
    EPI_T(et0);
    float sg[2] = {0.f, 0.f}, sgx[2] = {0.f, 0.f}, sx[2] = {0.f, 0.f};
    vm_wait<0>();  // the staged y tiles have landed
    auto pass1 = [&](f32x16 (&acc)[MT], int nt) {
        const int n = c0 + 32 * nt + l32;
        const float bv = a.bias ? a.bias[n] : 0.f;
        const float mu = a.bnb_mean[n], is = a.bnb_invstd[n], sc = a.bnb_scale[n], sh = a.bnb_shift[n];
        const __bf16* ys = reinterpret_cast<const __bf16*>(stg + nt * X6_STG_WAVE) + l32;
        auto part = [&](float d, float y) {
            const float gv = fmaf(y, sc, sh) > 0.f ? d : 0.f;
            const float xh = (y - mu) * is;
            sg[nt] += gv;
            sgx[nt] = fmaf(gv, xh, sgx[nt]);
            sx[nt] += xh;
        };
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            if (wm * MT + mt >= vh) break;  // uniform
            const __bf16* t16 = ys + mt * 1024;
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                float v0 = acc[mt][r] + bv, v1 = acc[mt][r + 1] + bv;
                pk_bf16(v0, v1, v0, v1);
                acc[mt][r] = v0;
                acc[mt][r + 1] = v1;
                part(v0, (float)t16[((r & 3) + 8 * (r >> 2) + 4 * h) * 32]);
                part(v1, (float)t16[(((r + 1) & 3) + 8 * ((r + 1) >> 2) + 4 * h) * 32]);
            }
            asm volatile("" ::: "memory");
        }
    };
    pass1(acc0, 0);
    pass1(acc1, 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // y reads done: the areas are free
    auto pk = [](float x, float y) {
        return (__builtin_bit_cast(unsigned, x) >> 16) | (__builtin_bit_cast(unsigned, y) & 0xffff0000u);
    };
    const int k = lane & 7;
    const float* const sk = (k < 4 ? stg : stg1) + 8 * (k & 3);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int py = wm * MT + mt;
        if (py >= vh) break;  // uniform
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const int p0 = (r & 3) + 8 * (r >> 2) + 4 * h;
            stg[p0 * P + l32] = acc0[mt][r];
            stg[(p0 + 1) * P + l32] = acc0[mt][r + 1];
            stg1[p0 * P + l32] = acc1[mt][r];
            stg1[(p0 + 1) * P + l32] = acc1[mt][r + 1];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const size_t rowb = (size_t)((b * a.H + ty0 + py) * a.W + tx0) * a.Cout + c0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int p = (lane >> 3) + 8 * j;
            const f32x4 lo = *reinterpret_cast<const f32x4*>(sk + p * P);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(sk + p * P + 4);
            const u32x4 w = {pk(lo.x, lo.y), pk(lo.z, lo.w), pk(hi.x, hi.y), pk(hi.z, hi.w)};
            __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(a.out0_16 + rowb + (size_t)p * a.Cout + 8 * k));
        }
        asm volatile("" ::: "memory");
    }
    EPI_T(et1);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        sg[nt] += __shfl_xor(sg[nt], 32, 64);
        sgx[nt] += __shfl_xor(sgx[nt], 32, 64);
        sx[nt] += __shfl_xor(sx[nt], 32, 64);
    }
    if (lane < 32) {
        const size_t S = WM * (size_t)a.ntiles, slot = WM * (size_t)tile + wm;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            const size_t n = c0 + 32 * nt + l32;
            a.bnb_part[(0 * (size_t)a.Cout + n) * S + slot] = sg[nt];
            a.bnb_part[(1 * (size_t)a.Cout + n) * S + slot] = sgx[nt];
            a.bnb_part[(2 * (size_t)a.Cout + n) * S + slot] = sx[nt];
        }
    }
    EPI_REC(et0, et1);
}

// Epilogue of the 16x16x32 form: acc[mt][nt] is D[oc][px] of m-tile mt (16 pixels:
// image row wm*4 + mt/2, columns (mt&1)*16 + 0..15) and n-tile nt (16 channels); lane
// (g, l) holds channels 4g..4g+3 of pixel l -> one 16-byte store per tile.  BatchNorm
// partials as x6_epilogue_wave (slot 2*tile + wm), reduced over the pixel lanes of
// each DPP row.  (A full-width specialisation as in x6_epilogue_wave measured neutral
// here -- its column guard is one branch per m-tile -- and spilled; profiles/r5f_ab_fullwidth_epilogue_x6.txt.)
template <int TH, int TW, int NWM = 2>
__device__ __forceinline__ void x6q_epilogue_wave(const ConvFwdArgs& a,
                                                  f32x4 (&acc)[TH * TW / 16 / NWM][2],
                                                  int tile, int b, int ty0, int tx0, int n0, int wm,
                                                  int wn) {
    static_assert((TH * TW == 256 || TH * TW == 128) && (TW == 32 || TW == 16),
                  "256- or 128-pixel tiles");
    constexpr int WR = TH / NWM;  // image rows of one wave (NWM pixel groups per tile)
    constexpr int MTW = TH * TW / 16 / NWM;  // m-tiles of one wave
    auto prow = [](int mt) { return TW == 32 ? mt >> 1 : mt; };
    auto pcol = [](int mt) { return TW == 32 ? (mt & 1) * 16 : 0; };
    const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
    const int vh = min(TH, a.H - ty0), vw = min(TW, a.W - tx0);
    float* out;
    int ostride, ocol0, oacc;
    if (n0 < a.split) {
        out = a.out0;
        ostride = a.split;
        ocol0 = n0;
        oacc = a.acc0;
    } else {
        out = a.out1;
        ostride = a.Cout - a.split;
        ocol0 = n0 - a.split;
        oacc = a.acc1;
    }
    const int c0 = wn * 32 + 4 * g;  // + 16 nt
    f32x4 bv[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
#ifdef X6Q_NOBIAS
        bv[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#else
        bv[nt] = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + n0 + c0 + 16 * nt)
                        : f32x4{0.f, 0.f, 0.f, 0.f};
#endif
    }
    f32x4 psum[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    // the stores of m-tiles [m0, m1)
    auto store_tiles = [&](auto accumulate, int m0, int m1) {
        constexpr bool ACC = decltype(accumulate)::value;
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt) {
            if (mt < m0 || mt >= m1) continue;
            const int py = wm * WR + prow(mt), px = pcol(mt) + l16;
            if (py >= vh) break;  // uniform
            const bool ok = px < vw;
            float* p = out + (size_t)((b * a.H + ty0 + py) * a.W + tx0 + px) * ostride + ocol0 + c0;
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                // scalar arithmetic throughout: packed f32 VALU (v_pk_*) beside the
                // partner waves' MFMAs costs more than it saves (MI355X_MICROARCH.md)
                f32x4 v;
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = acc[mt][nt][i] + bv[nt][i];
                acc[mt][nt] = v;
#ifdef X6Q_NOSTORE  // diagnostic build: no output stores (results are wrong)
                if (ok && v[0] == 12345.f) {
#else
                if (ok) {
#endif
                    f32x4* q = reinterpret_cast<f32x4*>(p + 16 * nt);
                    if constexpr (ACC) {
                        const f32x4 o = *q;
#pragma unroll
                        for (int i = 0; i < 4; ++i) v[i] += o[i];
                    }
                    // (plain: non-temporal here made the fp32 step 1.4 % slower -- the next
                    // layer reads this output -- profiles/r6f_ab_nontemporal_epilogue_stores.txt)
                    *q = v;
#pragma unroll
                    for (int i = 0; i < 4; ++i) psum[nt][i] += acc[mt][nt][i];
                }
            }
        }
    };
    const bool bnb = a.bnb_part != nullptr && !oacc;  // (the host refuses bnb + accumulate)
    EPI_T(et0);
    if (oacc) store_tiles(std::integral_constant<bool, true>{}, 0, MTW);
    else if (!bnb) store_tiles(std::integral_constant<bool, false>{}, 0, MTW);
    EPI_T(et1);
    if (bnb) {
        // BatchNorm-backward partials of the stored output da (the reduction of
        // ugpg_bn_relu_bwd, bn.hip bn_bwd_reduce_kernel, on the tile still in registers):
        // g = da*[scale*y+shift > 0], xhat = (y-mean)*invstd; per slot sum g, g*xhat, xhat
        f32x4 mu[2], is[2], sc[2], sh[2], sg[2], sgx[2], sx[2];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            const int c = n0 + c0 + 16 * nt;
            mu[nt] = *reinterpret_cast<const f32x4*>(a.bnb_mean + c);
            is[nt] = *reinterpret_cast<const f32x4*>(a.bnb_invstd + c);
            sc[nt] = *reinterpret_cast<const f32x4*>(a.bnb_scale + c);
            sh[nt] = *reinterpret_cast<const f32x4*>(a.bnb_shift + c);
            sg[nt] = sgx[nt] = sx[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        // per batch of m-tiles: the y loads go out first, the batch's output stores issue
        // while they are in flight, then the partials
        constexpr int YB = MTW < 4 ? MTW : 4;
#pragma unroll
        for (int m0 = 0; m0 < MTW; m0 += YB) {
            f32x4 yv[YB][2];
#pragma unroll
            for (int u = 0; u < YB; ++u) {
                const int mt = m0 + u;
                const int py = min(wm * WR + prow(mt), vh - 1), px = min(pcol(mt) + l16, vw - 1);
                const size_t yp = (size_t)((b * a.H + ty0 + py) * a.W + tx0 + px) * a.Cout + n0 + c0;
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) yv[u][nt] = a.bnb_y.ld4(yp + 16 * nt);
            }
            store_tiles(std::integral_constant<bool, false>{}, m0, m0 + YB);
#pragma unroll
            for (int u = 0; u < YB; ++u) {
                const int mt = m0 + u;
                if (wm * WR + prow(mt) < vh && pcol(mt) + l16 < vw) {
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const float y = yv[u][nt][i];
                            const float gv =
                                fmaf(y, sc[nt][i], sh[nt][i]) > 0.f ? acc[mt][nt][i] : 0.f;
                            const float xh = (y - mu[nt][i]) * is[nt][i];
                            sg[nt][i] += gv;
                            sgx[nt][i] = fmaf(gv, xh, sgx[nt][i]);
                            sx[nt][i] += xh;
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                sg[nt][i] = row16_sum(sg[nt][i]);
                sgx[nt][i] = row16_sum(sgx[nt][i]);
                sx[nt][i] = row16_sum(sx[nt][i]);
            }
        if (l16 < 8) {
            const int nt = l16 >> 2, i = l16 & 3;
            float v0 = 0.f, v1 = 0.f, v2 = 0.f;
#pragma unroll
            for (int t = 0; t < 8; ++t)
                if (t == l16) {
                    v0 = sg[t >> 2][t & 3];
                    v1 = sgx[t >> 2][t & 3];
                    v2 = sx[t >> 2][t & 3];
                }
            const size_t n = n0 + c0 + 16 * nt + i, S = NWM * (size_t)a.ntiles,
                         slot = NWM * (size_t)tile + wm;
            a.bnb_part[(0 * (size_t)a.Cout + n) * S + slot] = v0;
            a.bnb_part[(1 * (size_t)a.Cout + n) * S + slot] = v1;
            a.bnb_part[(2 * (size_t)a.Cout + n) * S + slot] = v2;
        }
        return;
    }
    if (a.stats == nullptr) return;
#ifdef X6Q_NOSTATS
    return;
#endif
    const int rows = min(max(vh - wm * WR, 0), WR);
    const float cnt = (float)(rows * vw);
    f32x4 mu[2], q[2];
    // the centring shift of the second moment: any value near the mean gives the same
    // M2 to rounding (the finalize merges (count, sum, M2) exactly), so one reciprocal
    // replaces eight fp32 divisions per wave and item
    const float rcnt = cnt > 0.f ? 1.f / cnt : 0.f;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            psum[nt][i] = row16_sum(psum[nt][i]);
            mu[nt][i] = psum[nt][i] * rcnt;
        }
        q[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
        if (wm * WR + prow(mt) >= vh) break;  // uniform
        if (pcol(mt) + l16 < vw) {
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float d = acc[mt][nt][i] - mu[nt][i];
                    q[nt][i] = fmaf(d, d, q[nt][i]);
                }
            }
        }
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) q[nt][i] = row16_sum(q[nt][i]);
    // lane l < 8 of each row writes channel 16*(l>>2) + 4g + (l&3)
    if (l16 < 8) {
        const int nt = l16 >> 2, i = l16 & 3;
        float sv = 0.f, qv = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (t == l16) {
                sv = psum[t >> 2][t & 3];
                qv = q[t >> 2][t & 3];
            }
        const size_t n = n0 + c0 + 16 * nt + i, S = NWM * (size_t)a.ntiles,
                     slot = NWM * (size_t)tile + wm;
        a.stats[(0 * (size_t)a.Cout + n) * S + slot] = cnt;
        a.stats[(1 * (size_t)a.Cout + n) * S + slot] = sv;
        a.stats[(2 * (size_t)a.Cout + n) * S + slot] = qv;
    }
    EPI_REC(et0, et1);
}

#if defined(X6R_CLOCK) || defined(X6R_STAMP) || defined(X6W_STAMP)
__device__ unsigned long long g_clk[8192];
#endif
#if defined(X6R_STAMP) || defined(X6W_STAMP)
// diagnostic build only: median over workgroups (16-slot records) of the loader waves'
// fraction of the main loop spent in vm_wait (out[0..2], per phase) and at barriers
// (out[3..5]); the first compute wave's fraction at barriers (out[6]) and in the
// per-item epilogue (out[7]); loop cycles per step of the compute wave (out[8]); cycles of
// the last epilogue's store phase (out[9]) and statistics phase (out[10]); the loader waves'
// fractions of the loop in halo stores (out[11]), weight-row DMA issue (out[12]) and halo
// loads + cursor advances (out[13])
extern "C" int ugpg_debug_stamps(double* out) {
    static unsigned long long h[8192];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_clk), sizeof(h)) != hipSuccess) return -1;
#ifdef X6R_STAMP
    static unsigned long long he[512 * 4];
    if (hipMemcpyFromSymbol(he, HIP_SYMBOL(g_epi), sizeof(he)) != hipSuccess) return -1;
#endif
    static double f[14][512];
    int n = 0;
    for (int i = 0; i < 512; ++i)
        if (h[16 * i] > 0) {
            const unsigned long long* r = h + 16 * i;
            for (int q = 0; q < 6; ++q) f[q][n] = (double)r[1 + q] / r[0];
            for (int q = 0; q < 3; ++q) f[11 + q][n] = (double)r[12 + q] / r[0];
            f[6][n] = r[8] ? (double)r[9] / r[8] : 0.0;
            f[7][n] = r[8] ? (double)r[10] / r[8] : 0.0;
            f[8][n] = r[11] ? (double)r[8] / r[11] : 0.0;
#ifdef X6R_STAMP
            f[9][n] = (double)he[4 * i];
            f[10][n] = (double)he[4 * i + 1];
#else
            f[9][n] = f[10][n] = 0.0;
#endif
            ++n;
        }
    for (int q = 0; q < 14; ++q) {
        std::sort(f[q], f[q] + n);
        out[q] = n ? f[q][n / 2] : 0.0;
    }
    return n;
}
#endif
#ifdef X6R_CLOCK
// diagnostic build only: per-workgroup (core cycles, 100 MHz ticks) of the main loop
extern "C" int ugpg_debug_clock(double* mhz) {
    static unsigned long long h[8192];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_clk), sizeof(h)) != hipSuccess) return -1;
    double r[4096];
    int n = 0;
    for (int i = 0; i < 4096; ++i)
        if (h[2 * i + 1] > 0) r[n++] = 100.0 * (double)h[2 * i] / (double)h[2 * i + 1];
    std::sort(r, r + n);
    *mhz = n ? r[n / 2] : 0.0;
    return n;
}
#endif
// THT: tile height; 256 / TWT (256-pixel items) by default, 8 with TWT = 16 for 128-pixel
// items (8 x 16) on 16-wide images, whose 256-pixel items would leave half of the CUs idle
// at bs16 (64 images' worth of 16 x 16 tiles x 8 column blocks = 128 items).  (Measured
// and dropped: two compute waves per SIMD, 512-pixel single-piece items, column-block-major
// item order.)
// RES (single-piece 256 x 64 items, K = 64, one column block): the weights of the whole
// launch -- 4 steps x 3 kernel rows, 72 KB -- stay resident in LDS, DMA'd once in the
// prologue; the loaders' steady state is halo loads and stores only (the row DMAs were 14-20 %
// of their loop: profiles/r7a stamps)
template <int NP, bool M16, int TWT = 32, int THT = 256 / TWT, bool XB16 = false, int NSLAB = 1,
          bool RES = false, int PAIR = 0>
__global__ void __launch_bounds__(8 * 64, 1) conv3x3_fwd_x6r_kernel(ConvFwdArgs a) {
    constexpr int NCW = 4;  // compute waves (one per SIMD) + 4 loader waves
    static_assert(!M16 || NP == 3, "the 16x16x32 form pairs the split-bf16 products");
    // XB16: every source is stored in bf16 only (single-piece form): one 16-byte halo load
    // per (pixel, 8 channels) instead of two
    static_assert(!XB16 || NP == 1, "bf16 sources only in the single-piece form");
    // 16-wide tiles: the 16x16x32 form, or (single piece) 8 x 16 items of a 16-wide image
    // whose 32-pixel MFMA tiles are two image rows (round 6)
    static_assert(TWT == 32 || (TWT == 16 && (M16 || (NP == 1 && THT == 8 && NSLAB == 1))),
                  "16-wide tiles");
    // items: 256 pixels (8 x 32, or 16 x 16 for 16-31 wide images in the 16x16x32 form;
    // 128 = 8 x 16 there too) x 64 output channels; the single-piece form also runs
    // 256 x 128 (NSLAB = 2 weight slabs of 64 columns) and 512 x 64 (16 x 32) items
    static_assert(THT * TWT == 256 || (THT * TWT == 128 && (M16 || NP == 1)) ||
                      (NP == 1 && THT * TWT == 512 && NSLAB == 1),
                  "item shapes");
    static_assert(NSLAB == 1 || (NP == 1 && THT * TWT == 256 && NSLAB == 2), "64 x NSLAB columns");
    constexpr int TW = TWT, TH = THT, BN = 64, BKC = 16, BNI = BN * NSLAB;
    // 32x32x16 form: the compute waves as WM (pixel rows) x WN (columns); each covers
    // MT 32-pixel image rows x NT 32-column n-tiles.  256 x 64 items: 2 x 2 waves of 4 x 1
    // tiles (an A fragment feeds one MFMA); 256 x 128 and 512 x 64 items: 4 x 2 tiles per
    // wave (each A fragment feeds two MFMAs, each B fragment four: 0.75 fragment reads per
    // MFMA instead of 1.25 -- the single-piece form's LDS read traffic set its pace)
    // MR: image rows per 32-pixel m-tile of the 32x32x16 form (2 for 16-wide tiles)
    constexpr int WM = M16 || TH * TW < 256 ? 2 : TH * TW / 128, WN = NCW / WM, MR = 32 / TW,
                  MT = M16 ? TH / 2 : TH * TW / (32 * WM), NT = M16 ? 1 : BNI / (32 * WN);
    static_assert(M16 || (WM * WN == NCW && NT >= 1 && MT * WM * 32 == TH * TW), "wave grid");
    // halo row pitch HS in 16-B pixel slots.  The single-piece 16-wide form's A fragment
    // is two image rows (lanes 0-15 / 16-31): a ds_read_b128 lane group {0-3,12-15,20-27}
    // then holds pixels 0-3, 12-15 of one row and 4-11 of the next, conflict-free only
    // when HS = 0 (mod 16) -- the dense pitch 18 made every A read 2-way in each group
    // (2.18 conflict cycles per LDS instruction, profiles/r7b_bf16_summary.md)
#ifndef X6R_W16_HS  // (A/B build: X6R_W16_HS=18, the dense pitch)
#define X6R_W16_HS 32
#endif
    constexpr int HWD = TW + 2, HS = TW == 16 && !M16 ? X6R_W16_HS : HWD;
    static_assert(HS >= HWD, "halo row pitch");
    constexpr int NHALO = (TH + 2) * HWD;                   // 340 / 324 halo pixels
    constexpr int NSPARE = (TH + 2) * HS;                   // the idle lanes' slot
    // spare slot NSPARE; plane pitch 348 = 4 (mod 8) for the 32x32 fragment pattern, 352
    // = 0 (mod 16) for the 16x16 one (ds_read_b128 lane groups, MI355X_MICROARCH.md §LDS)
    constexpr int NHP = M16 ? (NSPARE + 1 + 15) / 16 * 16 : NSPARE + 1 + (11 - NSPARE % 8) % 8;
    // (halo pixel, channel half) items: lane group i of 16 takes 16 consecutive pixels of
    // one half (i & 1), so each 8-lane group of a halo ds_write_b128 stores 128 contiguous
    // bytes of one plane -- conflict-free (the two halves of a pixel sit 352 vectors apart,
    // i.e. on the same banks; pairing them in one 8-lane group was a 2-way conflict on
    // every halo store: 0.35 conflict cycles per LDS instruction, profiles/r1i)
    constexpr int A_ITEMS = (NHALO + 15) / 16 * 32;         // 704 / 672 incl. idle lanes
    constexpr int A_PER = (A_ITEMS + 255) / 256;            // 3
    constexpr int A_VECS = 2 * NP * NHP;
    constexpr int R_VEC = NP * 2 * 3 * BN;                  // one kernel row of a 64-column slab
    constexpr int R_PER = (R_VEC + 255) / 256;
    constexpr int R_STR = NSLAB * R_VEC;                    // ring slot pitch: the item's slabs
    // weight rows DMA'd LA rows ahead of the row the compute waves read (ring NSLOT >=
    // LA + 1).  Three rows = two phases of flight cover the DMA latency when a phase holds
    // 3 x 6 split-bf16 MFMA groups; the single-piece form's phases are a sixth as long,
    // so it runs six rows (five phases) ahead in a ring of eight (6 KiB slots)
#ifndef X6R_NP1_LA
#define X6R_NP1_LA 6
#endif
#ifndef X6R_CTAB_MAX  // channels of both sources the single-piece LDS coefficient table holds
#define X6R_CTAB_MAX 2048
#endif
    // (the single-piece form's larger items have phases twice as long: three rows ahead)
    constexpr int LA = NP == 1 && TH * TW * NSLAB <= 256 ? X6R_NP1_LA : 3;
    static_assert(LA == 3 || LA == 6, "row lookahead: one or two steps");
    static_assert(!RES || (NP == 1 && NSLAB == 1 && TH * TW == 256), "resident weights: 256 x 64 single piece");
    constexpr int RES_NCH = 4;  // (the host launches RES for K = 64 only)
    // ring slot of row j = 3 step + ky: j % NSLOT, i.e. 3 (step % 4) + ky with RES
    constexpr int NSLOT = RES ? 3 * RES_NCH : LA == 3 ? 4 : 8;
    __shared__ __attribute__((aligned(16))) u32x4 smem[2 * A_VECS + NSLOT * R_STR + 1];
    // single-piece form: the activation coefficients of every input channel staged in LDS
    // once per launch, so the loaders' steady-state global instructions are halo loads and
    // weight DMAs only (that form is bound by its loaders' memory-instruction issue)
    constexpr bool CTAB = NP == 1;
    constexpr int CTAB_N = CTAB ? X6R_CTAB_MAX : 4;
    __shared__ __attribute__((aligned(16))) float ctab[2][CTAB_N];
    // the 32x32-form epilogue's per-wave staging of bf16-only outputs (x6_epilogue_wave)
    constexpr int OSTG_N = M16 ? 4 : NCW * NT * X6_STG_WAVE;
    __shared__ __attribute__((aligned(16))) float ostg[OSTG_N];
    u32x4* const Bring = smem + 2 * A_VECS;
    u32x4* const dummy = smem + 2 * A_VECS + NSLOT * R_STR;  // writes of idle lanes

    // the wave index in an SGPR: role, wave-grid position and staging addresses are
    // wave-uniform (scalar registers, scalar branches), not per-lane VGPR values
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool loader = wave >= NCW;
    const int NB = a.Cout / BNI;
    const int nitems = a.ntiles * NB;
    const int nslots = gridDim.x >> 3;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int iq = nitems >> 3, ir = nitems & 7;
    const int ibeg = xcd * iq + min(xcd, ir);
    const int iend = ibeg + iq + (xcd < ir ? 1 : 0);
    const int item0 = ibeg + slot;
    if (item0 >= iend) return;  // uniform per workgroup
    const int nchunk = a.Cin / BKC;
    const int total = (iend - item0 + nslots - 1) / nslots * nchunk;  // steps of this workgroup
    const int last = total - 1;
    const int tpi = a.tiles_x * a.tiles_y;

    struct Pos {
        int b, ty0, tx0, nb, tile;
    };
    auto pos_of = [&](int it) {
        Pos p;
        p.nb = it % NB;
        p.tile = it / NB;
        p.b = p.tile / tpi;
        const int trem = p.tile % tpi;
        p.ty0 = (trem / a.tiles_x) * TH;
        p.tx0 = (trem % a.tiles_x) * TW;
        return p;
    };

    if (loader) {
        // ------------------------------------------------------------ loader waves
        // Halo of step s: loaded into register set s & 1 (f32, with its activation
        // coefficients) three steps ahead, written (activated, split) into A buffer s & 1
        // during phases 0-1 of step s-1.  Weight rows: LDS-DMA, see below.
        const int lt = tid - NCW * 64;
        const int hhl = (lt >> 4) & 1;  // channel half of this lane (same for all its items)
        auto item_px = [](int idx) { return (idx >> 5) * 16 + (idx & 15); };
        constexpr int LPV = XB16 ? 1 : 2;  // global loads per halo vector
        f32x4 ra[2][A_PER][LPV];
        unsigned avalid[2] = {0u, 0u};
        Act4 r0[2], r1[2];
        float lo[2] = {0.f, 0.f};
        bool b16[2] = {false, false};
        // cursor over loader steps (clamped to the last one): chunk, item, column block
        // and tile position, advanced without divisions except at item changes
        // per-lane halo pixel offsets (row, column within the halo) of the A_PER vectors
        int hy[A_PER], hx[A_PER];
#pragma unroll
        for (int v = 0; v < A_PER; ++v) {
            const int hp = item_px(lt + v * 256);
            hy[v] = hp < NHALO ? hp / HWD : -(1 << 20);  // never inside the image
            hx[v] = hp % HWD;
        }
        // the halo cursor also carries, per item, each vector's (clamped) image pixel
        // index and whether it lies inside the image: a step then addresses its loads
        // with one multiply-add per vector
        struct Cur {
            int s, c, itm, nb;
            Pos p;
            int pix[A_PER];
            unsigned pok;
        };
        auto locate = [&](Cur& q) {
            unsigned ok = 0;
#pragma unroll
            for (int v = 0; v < A_PER; ++v) {
                const int gy = q.p.ty0 - 1 + hy[v], gx = q.p.tx0 - 1 + hx[v];
                ok |= (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W ? 1u : 0u) << v;
                const int cy = min(max(gy, 0), a.H - 1), cx = min(max(gx, 0), a.W - 1);
                q.pix[v] = (q.p.b * a.H + cy) * a.W + cx;
            }
            q.pok = ok;
        };
        auto cur_at = [&](int s, bool halo) {
            Cur q;
            q.s = min(s, last);
            q.c = q.s % nchunk;
            q.itm = item0 + (q.s / nchunk) * nslots;
            q.nb = q.itm % NB;
            q.p = pos_of(q.itm);
            if (halo) locate(q);
            return q;
        };
        auto advance = [&](Cur& q, bool halo) {
            if (q.s >= last) return;
            ++q.s;
            if (++q.c == nchunk) {
                q.c = 0;
                q.itm += nslots;
                q.nb = q.itm % NB;
                q.p = pos_of(q.itm);
                if (halo) locate(q);
            }
        };
        auto load_halo = [&](const Cur& q, auto S, auto TABC) {
            constexpr int st = decltype(S)::value;
            constexpr bool TAB = decltype(TABC)::value;
            const int c = q.c;
            const int cb0 = c * BKC;
            const bool second = cb0 >= a.C0;
            const float* src = second ? a.src1 : a.src0;
            // single-piece form: a source's bf16 copy is read instead (half the bytes; the
            // second load repeats the first address, so the load count stays fixed)
            const __bf16* s16 = NP == 1 ? (second ? a.src1_16 : a.src0_16) : nullptr;
            b16[st] = XB16 || s16 != nullptr;
            const float* sc = second ? a.sc1 : a.sc0;
            const float* sh = second ? a.sh1 : a.sh0;
            const int Cs = second ? a.C1 : a.C0;
            const int cb = second ? cb0 - a.C0 : cb0;
            const bool aon = sc != nullptr;
            const float* scp = aon ? sc : g_act_ones;  // identity coefficients without activation
            const float* shp = aon ? sh : g_act_zeros;
            lo[st] = aon ? 0.f : -INFINITY;
            // an 8-channel source is zero-extended to the 16-channel chunk
            const bool cok = cb + hhl * 8 < Cs;
            const int cc = cb + (cok ? hhl * 8 : 0);
            if constexpr (TAB) {
                const int tc = (second ? a.C0 : 0) + cc;
                r0[st].s = *reinterpret_cast<const f32x4*>(&ctab[0][tc]);
                r0[st].h = *reinterpret_cast<const f32x4*>(&ctab[1][tc]);
                r1[st].s = *reinterpret_cast<const f32x4*>(&ctab[0][tc + 4]);
                r1[st].h = *reinterpret_cast<const f32x4*>(&ctab[1][tc + 4]);
            } else {
                r0[st].s = gld16(scp + cc);
                r0[st].h = gld16(shp + cc);
                r1[st].s = gld16(scp + cc + 4);
                r1[st].h = gld16(shp + cc + 4);
            }
#pragma unroll
            for (int v = 0; v < A_PER; ++v) {
                const size_t off = (size_t)q.pix[v] * Cs + cc;
                if constexpr (XB16) {
                    ra[st][v][0] = gld16(s16 + off);
                } else {
                    const void* g0 = s16 ? static_cast<const void*>(s16 + off)
                                         : static_cast<const void*>(src + off);
                    const void* g1 = s16 ? g0 : static_cast<const void*>(src + off + 4);
                    ra[st][v][0] = gld16(g0);
                    ra[st][v][LPV - 1] = gld16(g1);
                }
            }
            avalid[st] = cok ? q.pok : 0u;
        };
        constexpr int HALO_LOADS = (CTAB ? 0 : 4) + LPV * A_PER;  // global loads per loop halo
        auto store_halo = [&](int k, auto S, int v0, int v1) {
            constexpr int st = decltype(S)::value;
            u32x4* As = smem + (k & 1) * A_VECS;
            if constexpr (NP == 1) {
                if (b16[st] && !(lo[st] > -INFINITY)) {
                    // (uniform) a bf16 source without activation (a data gradient's dy, an Up
                    // conv's upsampled half): its 8 bf16 are already the single piece -- the
                    // bits go to LDS as they are (no widen / identity affine / round trip)
#pragma unroll
                    for (int v = v0; v < v1; ++v) {
                        const int hp = item_px(lt + v * 256);
                        const bool ok = (avalid[st] >> v) & 1u;
                        u32x4 w = __builtin_bit_cast(u32x4, ra[st][v][0]);
#pragma unroll
                        for (int i = 0; i < 4; ++i) w[i] = ok ? w[i] : 0u;
                        const int hl = hp < NHALO ? (hp / HWD) * HS + hp % HWD : NSPARE;
                        As[hhl * NHP + hl] = w;
                    }
                    return;
                }
            }
#pragma unroll
            for (int v = v0; v < v1; ++v) {
                const int hp = item_px(lt + v * 256), hh = hhl;
                f32x4 raw0 = ra[st][v][0], raw1 = ra[st][v][LPV - 1];
                if (NP == 1 && b16[st]) {  // 8 bf16 in the first load: widen (exact)
                    const u32x4 w = __builtin_bit_cast(u32x4, raw0);
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        raw0[2 * i] = __uint_as_float(w[i] << 16);
                        raw0[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
                        raw1[2 * i] = __uint_as_float(w[2 + i] << 16);
                        raw1[2 * i + 1] = __uint_as_float(w[2 + i] & 0xffff0000u);
                    }
                }
                const f32x4 lo4 = act_floor4(raw0, r0[st], lo[st]),
                            hi4 = act_floor4(raw1, r1[st], lo[st]);
                const bool ok = (avalid[st] >> v) & 1u;
                u32x4 pc[NP];
                if constexpr (NP == 1) {
                    // one piece: zero the four packed words instead of the eight floats
                    const f32x8 x = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
                    split_n<NP>(x, pc);
#pragma unroll
                    for (int i = 0; i < 4; ++i) pc[0][i] = ok ? pc[0][i] : 0u;
                } else {
                    const f32x8 x = {ok ? lo4.x : 0.f, ok ? lo4.y : 0.f, ok ? lo4.z : 0.f,
                                     ok ? lo4.w : 0.f, ok ? hi4.x : 0.f, ok ? hi4.y : 0.f,
                                     ok ? hi4.z : 0.f, ok ? hi4.w : 0.f};
                    split_n<NP>(x, pc);
                }
                const int hl = hp < NHALO ? (hp / HWD) * HS + hp % HWD : NSPARE;
#pragma unroll
                for (int q = 0; q < NP; ++q) As[(q * 2 + hh) * NHP + hl] = pc[q];
            }
        };
        using Set0 = std::integral_constant<int, 0>;
        using Set1 = std::integral_constant<int, 1>;
        // weight row j -> ring slot j % 4 by LDS-DMA: 16 B per lane, each wave-instruction
        // one contiguous KiB of the slot; rounds of 256 vectors, the last round's
        // missing waves repeat a present wave's copy (identical bytes, same place)
        constexpr int R_LASTW = (R_VEC - (R_PER - 1) * 256) / 64;  // waves with work in the last round
        static_assert(R_VEC % 64 == 0, "whole wave-instructions");
        const int lw = lt >> 6;
        auto dma_row = [&](const Cur& q, int ky, int slot) {
#pragma unroll
            for (int sb = 0; sb < NSLAB; ++sb) {
                const u32x4* ws = static_cast<const u32x4*>(a.wpk) +
                                  (((size_t)(q.nb * NSLAB + sb) * nchunk + q.c) * 3 + ky) * R_VEC;
                u32x4* Bs = Bring + slot * R_STR + sb * R_VEC;
#ifdef X6R_DMA_PERBLOCK  // A/B build: one M0 setting per block, blocks strided by wave
#pragma unroll
                for (int v = 0; v < R_PER; ++v) {
                    const int base = v * 256 + (v + 1 < R_PER ? lw : lw % R_LASTW) * 64;
                    glds16(ws + base + lane, Bs + base);
                }
#else
                // wave lw copies R_PER consecutive blocks of the row (the last wave's run
                // ends at the row's end, repeating blocks of the wave before it: identical
                // bytes to the same place), in runs of at most four blocks per M0 setting
                constexpr int NB = R_VEC / 64;
                const int b0 = min(lw * R_PER, NB - R_PER) * 64;
                glds16_run<(R_PER < 4 ? R_PER : 4)>(ws + b0 + lane, Bs + b0);
                if constexpr (R_PER > 4) glds16_run<R_PER - 4>(ws + b0 + 256 + lane, Bs + b0 + 256);
#endif
            }
        };
        // prologue: step 0 in LDS (halo buffer 0, rows 0-2), halos 1 and 2 in registers
        using TabOff = std::integral_constant<bool, false>;
        using TabOn = std::integral_constant<bool, CTAB>;
        if constexpr (CTAB) {
            // plain (tracked) loads, before any untracked one: hipcc's own waits retire them
            for (int i = lt * 4; i < a.C0 + a.C1; i += 256 * 4) {
                const bool s1 = i >= a.C0;
                const int c = s1 ? i - a.C0 : i;
                const float* scx = s1 ? a.sc1 : a.sc0;
                const float* shx = s1 ? a.sh1 : a.sh0;
                const f32x4 vs = scx ? *reinterpret_cast<const f32x4*>(scx + c) : f32x4{1.f, 1.f, 1.f, 1.f};
                const f32x4 vh = scx ? *reinterpret_cast<const f32x4*>(shx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
                *reinterpret_cast<f32x4*>(&ctab[0][i]) = vs;
                *reinterpret_cast<f32x4*>(&ctab[1][i]) = vh;
            }
        }
        {
            const Cur q0 = cur_at(0, true);
            load_halo(q0, Set0{}, TabOff{});
            vm_wait<0>();
            store_halo(0, Set0{}, 0, A_PER);
            dma_row(q0, 0, 0);
            dma_row(q0, 1, 1);
            dma_row(q0, 2, 2);
            if constexpr (RES) {  // every row of the launch (one column block, 4 steps)
#pragma unroll
                for (int c = 1; c < RES_NCH; ++c) {
                    const Cur qc = cur_at(c, false);
                    dma_row(qc, 0, 3 * c);
                    dma_row(qc, 1, 3 * c + 1);
                    dma_row(qc, 2, 3 * c + 2);
                }
            } else if constexpr (LA == 6) {
                const Cur q1 = cur_at(1, false);
                dma_row(q1, 0, 3);
                dma_row(q1, 1, 4);
                dma_row(q1, 2, 5);
            }
            load_halo(cur_at(1, true), Set1{}, TabOff{});
            load_halo(cur_at(2, true), Set0{}, TabOff{});
            vm_wait<0>();
        }
        lds_barrier();
        Cur cw = cur_at(LA / 3, false), ch = cur_at(3, true);  // weight rows of step k+LA/3, halo of step k+3
        int sl = LA % NSLOT;                      // ring slot of row 3k+LA
        // Phase ph of step k DMAs row j = 3(k+1)+ph into the slot of row j-4 (read in
        // the phase before, whose MFMAs consumed it before that phase's barrier) and
        // retires the previous phase's row before its own closing barrier, so every row
        // has about two phases of flight and is read one phase after that barrier.
        // Phases 0-1 write halo(k+1) (the compute waves first read it in phase 2), then
        // phase 2 reloads the freed register set with halo(k+3).  vmcnt counts the
        // loader's loads and DMAs together, in issue order: retiring a row retires every
        // older halo load too.
        // loads per weight row (none in the loop with resident weights) / halo
        constexpr int R = RES ? 0 : NSLAB * R_PER, H = HALO_LOADS;
        constexpr int HA = (A_PER + 1) / 2;  // halo vectors written in phase 0
#ifdef X6R_STAMP
        // diagnostic build: loader cycles spent waiting for global loads / at barriers
        unsigned long long st_vm[3] = {0, 0, 0}, st_bar[3] = {0, 0, 0};
        unsigned long long st_sh = 0, st_dma = 0, st_lh = 0;  // halo stores, row DMAs, halo loads
        const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
#define ST_WAIT(acc, stmt)                                          \
    {                                                               \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        stmt;                                                       \
        acc += __builtin_amdgcn_s_memtime() - t_;                   \
    }
#else
#define ST_WAIT(acc, stmt) stmt
#endif
#if defined(X6R_NODMA) || defined(X6R_NOHALO)
// these builds drop loads under the counted vm waits, so a wait can leave a load in flight
// past the point where hipcc reuses its destination register (an address register: a GPU
// memory fault, seen with the six-row lookahead); audit the build before running one
#error "stream-removal diagnostic builds are unsafe with counted vm waits (see comment)"
#endif
#ifdef X6R_NODMA  // diagnostic builds: drop a load stream (results are wrong)
#define dma_row(...) ((void)0)
#endif
#ifdef X6R_NOHALO
#define load_halo(...) ((void)0)
#endif
        auto step = [&](int k, auto S) {  // S = set of halo(k+1); rows j = 3k + LA + ph
            // Each phase retires row 3k+ph+2 (read from the next phase on).  LA = 6: the
            // loads issued after that row are the next four rows plus one or two halo
            // batches, and phase 0 first retires halo(k+1) (issued right after row 3k+2)
            // before writing it.
            // phase 0
            if constexpr (!RES) ST_WAIT(st_dma, dma_row(cw, 0, sl));
            if constexpr (LA == 3) {
                ST_WAIT(st_sh, store_halo(k + 1, S, 0, HA));
                ST_WAIT(st_vm[0], vm_wait<H + R>());  // row j-1
            } else {
                ST_WAIT(st_vm[0], vm_wait<4 * R + H>());  // halo(k+1), row 3k+2
                ST_WAIT(st_sh, store_halo(k + 1, S, 0, HA));
            }
            ST_WAIT(st_bar[0], lds_barrier());
            // phase 1
            if constexpr (!RES) ST_WAIT(st_dma, dma_row(cw, 1, (sl + 1) % NSLOT));
            ST_WAIT(st_sh, store_halo(k + 1, S, HA, A_PER));
            if constexpr (LA == 3) {
                ST_WAIT(st_vm[1], vm_wait<R>());  // row j (and halo(k+2))
            } else {
                ST_WAIT(st_vm[1], vm_wait<4 * R + H>());  // row 3k+3
            }
            ST_WAIT(st_bar[1], lds_barrier());
            // phase 2
            if constexpr (!RES) ST_WAIT(st_dma, dma_row(cw, 2, (sl + 2) % NSLOT));
            ST_WAIT(st_lh, load_halo(ch, S, TabOn{}); advance(cw, false); advance(ch, true));
            sl = (sl + 3) % NSLOT;
            if constexpr (LA == 3) {
                ST_WAIT(st_vm[2], vm_wait<R + H>());  // row j+1
            } else {
                ST_WAIT(st_vm[2], vm_wait<4 * R + 2 * H>());  // row 3k+4
            }
            // phase 2 writes no LDS (its DMA completions are the vmcnt wait above): no
            // lgkmcnt(0) before this barrier, so the coefficient-table reads of load_halo
            // (consumed by the next phase-0 halo stores) stay in flight across it
            ST_WAIT(st_bar[2], read_barrier());
        };
        static_assert(RES || ((NSLOT & (NSLOT - 1)) == 0 && NSLOT >= LA + 1), "ring slot arithmetic");
        for (int k = 0; k < total; k += 2) {
            step(k, Set1{});
            if (k + 1 < total) step(k + 1, Set0{});
        }
#undef dma_row
#undef load_halo
#undef ST_WAIT
        vm_wait<0>();  // no load outlives the workgroup (nothing may run before this wait:
                       // the last loads' destination registers are dead to the compiler)
#ifdef X6R_STAMP
        if (tid == NCW * 64 && blockIdx.x < 512) {
            g_clk[16 * blockIdx.x] = __builtin_amdgcn_s_memtime() - st_t0;
            for (int q = 0; q < 3; ++q) {
                g_clk[16 * blockIdx.x + 1 + q] = st_vm[q];
                g_clk[16 * blockIdx.x + 4 + q] = st_bar[q];
            }
            g_clk[16 * blockIdx.x + 12] = st_sh;
            g_clk[16 * blockIdx.x + 13] = st_dma;
            g_clk[16 * blockIdx.x + 14] = st_lh;
        }
#endif
        return;
    }
#ifdef X6R_STAMP
    // diagnostic build: the compute waves' cycles at barriers and in the epilogue
    unsigned long long cs_bar = 0, cs_epi = 0;
    const unsigned long long cs_t0 = __builtin_amdgcn_s_memtime();
#define CS_WAIT(acc, stmt)                                          \
    {                                                               \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        stmt;                                                       \
        acc += __builtin_amdgcn_s_memtime() - t_;                   \
    }
#define CS_STORE()                                                          \
    if (tid == 0 && blockIdx.x < 512) {                                     \
        g_clk[16 * blockIdx.x + 8] = __builtin_amdgcn_s_memtime() - cs_t0; \
        g_clk[16 * blockIdx.x + 9] = cs_bar;                                \
        g_clk[16 * blockIdx.x + 10] = cs_epi;                               \
        g_clk[16 * blockIdx.x + 11] = total;                                \
    }
#else
#define CS_WAIT(acc, stmt) stmt
#define CS_STORE()
#endif

    // ---------------------------------------------------------------- compute waves
    const int wm = wave / WN, wn = wave % WN;
    if constexpr (M16) {
        // 16x16x32 form: D[oc][px] = W x A with the split-bf16 products paired along k:
        // k-groups (lanes 16g..16g+15) 0,1 = channels 0-7, 8-15 of one piece, 2,3 of
        // another, so  W00.A01 = b0a0 + b0a1,  W11.A01 = b1a0 + b1a1,  W20.A02 = b2a0 + b0a2
        // (all six products, three MFMAs per 16x16 tile and tap).  A "unit" is a pair of
        // m-tiles (one image row, 32 pixels) of one tap: 4 A fragments, 12 MFMAs on four
        // accumulators; the next unit's A fragments and, spread over the tap, the next
        // tap's six W fragments are read while it runs.
        const int g = lane >> 4, l16 = lane & 15;
        // NWM pixel groups per tile: a wave covers TH/NWM image rows = MTW m-tiles of 16
        // pixels (row mt/2, columns 16(mt&1).. for 8 x 32 tiles; row mt for 16 x 16 tiles)
        constexpr int NWM = NCW / 2, MTW = TH * TW / 16 / NWM, URT = MTW / 2, UPS = 9 * URT;
        static_assert(URT >= 1, "a wave needs at least one m-tile pair");
        constexpr int WPU = (6 + URT - 1) / URT;  // next tap's W fragments read per unit
        const int a01 = g * NHP + wm * (TH / NWM) * HS + l16;
        const int a02 = ((g >> 1) * 4 + (g & 1)) * NHP + wm * (TH / NWM) * HS + l16;
        const int bo = (g & 1) * 3 * BN + wn * 32 + l16;
        const int wq[3] = {bo + 4 * 3 * BN * (g < 2 ? 1 : 0), bo + 2 * 3 * BN, bo};  // W20, W11, W00
        f32x4 acc[MTW][2];
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#ifndef X6Q_DEPTH
#define X6Q_DEPTH 1
#endif
        // A fragments are read DA units ahead (a ring of DA+1 must divide the step's units)
        constexpr int DA = UPS % (X6Q_DEPTH + 1) == 0 ? X6Q_DEPTH : 2;
        static_assert(UPS % (DA + 1) == 0, "unit ring must divide a step");
        u32x4 fa[DA + 1][2][2];  // [unit % (DA+1)][m-tile of the pair][A02, A01]
        u32x4 fw[3][3][2];     // [tap % 3 (9 taps per step)][W20, W11, W00][nt]
        auto lda = [&](const u32x4* As, int t, int r, u32x4 (&f)[2][2]) {
            const int ky = t / 3, kx = t % 3;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int o = TW == 32 ? (r + ky) * HS + kx + 16 * h : (2 * r + h + ky) * HS + kx;
                f[h][0] = As[a02 + o];
                f[h][1] = As[a01 + o];
            }
        };
        auto ldw = [&](const u32x4* Bs, int kx, int e, u32x4 (&f)[3][2]) {
            f[e >> 1][e & 1] = Bs[wq[e >> 1] + kx * BN + 16 * (e & 1)];
        };
        lds_barrier();  // step 0 staged
#ifdef X6R_CLOCK
        const unsigned long long clk_t0 = __builtin_amdgcn_s_memtime(),
                                 clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
        int cc = 0, item = item0;
        Pos cp = pos_of(item0);
#pragma unroll
        for (int uu = 0; uu < DA; ++uu) lda(smem, uu / URT, uu % URT, fa[uu]);
#pragma unroll
        for (int e = 0; e < 6; ++e) ldw(Bring, 0, e, fw[0]);
        for (int k = 0; k < total; ++k) {
            const u32x4* Ac = smem + (k & 1) * A_VECS;
            const u32x4* An = smem + ((k + 1) & 1) * A_VECS;
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int tn = t + 1 < 9 ? t + 1 : 0;  // next tap (of this step or the next)
                const u32x4* Bn = Bring + ((3 * k + (t + 1) / 3) % NSLOT) * R_STR;
#pragma unroll
                for (int r = 0; r < URT; ++r) {
                    const int u = t * URT + r;
                    // next unit's A fragments, then (spread over the tap) next tap's W
                    const int un = u + DA;
                    if (un < UPS) lda(Ac, un / URT, un % URT, fa[un % (DA + 1)]);
                    else lda(An, (un - UPS) / URT, (un - UPS) % URT, fa[un % (DA + 1)]);
                    constexpr int NWR = 0;
                    int nw = NWR;
#pragma unroll
                    for (int j = 0; j < WPU; ++j)
                        if (r * WPU + j < 6) {
                            ldw(Bn, tn % 3, r * WPU + j, fw[(t + 1) % 3]);
                            ++nw;
                        }
                    const u32x4(&A)[2][2] = fa[u % (DA + 1)];
                    const u32x4(&W)[3][2] = fw[t % 3];
#pragma unroll
                    for (int e = 0; e < 3; ++e)
#pragma unroll
                        for (int h = 0; h < 2; ++h)
#pragma unroll
                            for (int nt = 0; nt < 2; ++nt)
                                acc[2 * r + h][nt] =
                                    mfma16x16(W[e][nt], A[h][e == 0 ? 0 : 1], acc[2 * r + h][nt]);
#pragma unroll
                    for (int i = 0; i < 12; ++i) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                        if (i < 4 + nw) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (t % 3 == 2) CS_WAIT(cs_bar, read_barrier());
            }
            if (++cc == nchunk) {
                CS_WAIT(cs_epi, (x6q_epilogue_wave<TH, TW, NWM>(a, acc, cp.tile, cp.b, cp.ty0, cp.tx0,
                                                                cp.nb * BN, wm, wn)));
                cc = 0;
                item += nslots;
                if (item < iend) cp = pos_of(item);
#pragma unroll
                for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
#ifdef X6R_CLOCK
        if (tid == 0 && blockIdx.x < 4096) {
            g_clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - clk_t0;
            g_clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - clk_r0;
        }
#endif
        CS_STORE();
        return;
    } else {
    // acc[nt][mt]: n-tile nt (columns (wn*NT + nt)*32 of the item) of m-tile mt (image row
    // wm*MT + mt of the item)
    f32x16 acc[NT][MT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[nt][mt][r] = 0.f;
    const int hl = lane >> 5;
    // + MR*mt*HS + ky*HS + kx (16-wide tiles: lanes 16-31 read the m-tile's second row)
    const int aoff = TW == 32 ? hl * NHP + (wm * MT) * HS + (lane & 31)
                              : hl * NHP + (wm * MT * MR + ((lane & 31) >> 4)) * HS + (lane & 15);
    // n-tile nt of this wave: 32 columns of the ring slot's slab (wn*NT + nt) / 2 (the
    // wave's first column (wn*NT)*32 is a multiple of 64 when NT = 2)
    const int boff0 = (NT == 1 ? wn * 32 : wn * (R_VEC * NT / 2)) + hl * 3 * BN + (lane & 31);
    auto boff = [&](int nt) { return boff0 + (nt / 2) * R_VEC + (nt % 2) * 32; };
    auto ldfrag = [&](const u32x4* As, const u32x4* Bs, int ky, int kx, u32x4 (&af)[MT][NP],
                      u32x4 (&bf)[NT][NP]) {
#pragma unroll
        for (int q = 0; q < NP; ++q) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) af[mt][q] = As[q * 2 * NHP + aoff + (MR * mt + ky) * HS + kx];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) bf[nt][q] = Bs[q * 2 * 3 * BN + boff(nt) + kx * BN];
        }
    };
    // Every weight row a phase reads was completed a full phase earlier (the ring runs
    // one step ahead), so the fragments of the next phase's first tap are read BEFORE
    // the phase's barrier: the barriers only order the loaders' overwrites and expose
    // no LDS latency inside a step.
    // single-piece pipeline state: fragments read PD taps ahead into a ring of 3 sets
    // (9 taps per step: the set of a tap is t % 3 in every step).  Two taps ahead where a
    // tap is 4 MFMAs; one where it is 8 (whose 256 cycles cover the reads, and whose
    // 128 accumulator registers leave room for only two sets in flight)
    constexpr int PD = NT == 1 ? 2 : 1;
    u32x4 fa1[3][MT][NP], fb1[3][NT][NP];
    auto ldfrag1 = [&](int kk, int t, u32x4 (&af)[MT][NP], u32x4 (&bf)[NT][NP]) {
        const int ky = t / 3, kx = t % 3;
        ldfrag(smem + (kk & 1) * A_VECS, Bring + ((3 * kk + ky) % NSLOT) * R_STR, ky, kx, af, bf);
    };
    lds_barrier();  // step 0 staged
#ifdef X6R_CLOCK
    const unsigned long long clk_t0 = __builtin_amdgcn_s_memtime(),
                             clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
    int cc = 0, item = item0;
    Pos cp = pos_of(item0);
    // the wave's staging: NT areas of X6_STG_WAVE floats at ostg + (wave * NT + nt) * X6_STG_WAVE
    if constexpr (NP == 1) {
#pragma unroll
        for (int t = 0; t < PD; ++t) ldfrag1(0, t, fa1[t], fb1[t]);
    }
    for (int k = 0; k < total; ++k) {
        const u32x4* Ac = smem + (k & 1) * A_VECS;
        if constexpr (NP == 1) {
            // the item's last step: its BatchNorm-backward y tile (bf16) goes to the staging
            // area now, so the epilogue finds it landed
            if (cc == nchunk - 1 && a.bnb_part && a.bnb_y.h) {
                if constexpr (TW == 16) {  // (the epilogue's 32-wide view, below)
                    ConvFwdArgs av = a;
                    av.H = a.H / 2;
                    av.W = 32;
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        x6_dma_bnb_y<TH / 2, 32, MT>(av, cp.b, cp.ty0 / 2, 0,
                                                     cp.nb * BNI + (wn * NT + nt) * 32, wm,
                                                     ostg + (wave * NT + nt) * X6_STG_WAVE);
                } else {
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        x6_dma_bnb_y<TH, TW, MT>(a, cp.b, cp.ty0, cp.tx0,
                                                 cp.nb * BNI + (wn * NT + nt) * 32, wm,
                                                 ostg + (wave * NT + nt) * X6_STG_WAVE);
                }
            }
            // single piece: the reads run PD taps ahead, across the step boundary (the next
            // step's first taps are read in phase 2: halo(k+1) and row 3k+3 are visible there)
#pragma unroll
            for (int t = 0; t < 9; ++t) {
              if constexpr (NT == 2) {
                // 4 x 2 tiles, one tap ahead, m-tile-major MFMA order: the next tap's B
                // fragments first, then after each m-tile's two MFMAs its next A fragment
                // (into the register its current one frees), so 36 fragment registers are
                // live instead of 48.  The item's last tap prefetches nothing across the
                // epilogue; the step's last tap reads after its MFMAs (before the barrier).
                const int tn = (t + 1) % 3;
                const u32x4* An = smem + ((t + 1 < 9 ? k : k + 1) & 1) * A_VECS;
                const u32x4* Bn = Bring + ((3 * (t + 1 < 9 ? k : k + 1) + ((t + 1) % 9) / 3) % NSLOT) * R_STR;
                const int kyn = ((t + 1) % 9) / 3, kxn = (t + 1) % 3;
                auto ldA = [&](int mt) {
#pragma unroll
                    for (int q = 0; q < NP; ++q)
                        fa1[tn][mt][q] = An[q * 2 * NHP + aoff + (MR * mt + kyn) * HS + kxn];
                };
                auto ldB = [&](int nt) {
#pragma unroll
                    for (int q = 0; q < NP; ++q)
                        fb1[tn][nt][q] = Bn[q * 2 * 3 * BN + boff(nt) + kxn * BN];
                };
                if (t < 8) {
                    ldB(0);
                    ldB(1);
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        acc[0][mt] = mfma_xn<NP>(fa1[t % 3][mt], fb1[t % 3][0], acc[0][mt]);
                        acc[1][mt] = mfma_xn<NP>(fa1[t % 3][mt], fb1[t % 3][1], acc[1][mt]);
                        ldA(mt);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // B reads
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMAs
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // A read
                    }
                    __builtin_amdgcn_sched_barrier(0);
                } else {
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        acc[0][mt] = mfma_xn<NP>(fa1[t % 3][mt], fb1[t % 3][0], acc[0][mt]);
                        acc[1][mt] = mfma_xn<NP>(fa1[t % 3][mt], fb1[t % 3][1], acc[1][mt]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (cc != nchunk - 1) {
                        ldB(0);
                        ldB(1);
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt) ldA(mt);
                    }
                }
                if (t % 3 == 2) CS_WAIT(cs_bar, read_barrier());
                continue;
              }
                if (t + PD < 9) ldfrag1(k, t + PD, fa1[(t + PD) % 3], fb1[(t + PD) % 3]);
                else ldfrag1(k + 1, t + PD - 9, fa1[(t + PD) % 3], fb1[(t + PD) % 3]);
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
                        acc[nt][mt] = mfma_xn<NP>(fa1[t % 3][mt], fb1[t % 3][nt], acc[nt][mt]);
                constexpr int NM = MT * NT, NR = MT + NT;
#pragma unroll
                for (int i = 0; i < NM; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                    if (i < NR) {
                        if (NR > NM && i == 0)
                            __builtin_amdgcn_sched_group_barrier(0x100, NR - NM + 1, 0);
                        else
                            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                if (t % 3 == 2) CS_WAIT(cs_bar, read_barrier());
            }
        } else {
        u32x4 fa[2][MT][NP], fb[2][NT][NP];
        ldfrag(Ac, Bring + ((3 * k) % NSLOT) * R_STR, 0, 0, fa[0], fb[0]);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            if (t + 1 < 9) {
                const int ky1 = (t + 1) / 3, kx1 = (t + 1) % 3;
                ldfrag(Ac, Bring + ((3 * k + ky1) % NSLOT) * R_STR, ky1, kx1, fa[(t + 1) & 1],
                       fb[(t + 1) & 1]);
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    acc[nt][mt] = mfma_xn<NP>(fa[t & 1][mt], fb[t & 1][nt], acc[nt][mt]);
            // the next tap's fragment reads go out one per MFMA gap from the start of
            // this tap's MFMAs (fresh registers, landed long before their use)
            constexpr int NM = MT * NT * (NP == 3 ? 6 : 1), NR = (MT + NT) * NP;
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                     // MFMA
                if (t + 1 < 9 && i < NR) {
                    if constexpr (NR <= NM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    else __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // taps do not mix
            if (t % 3 == 2) CS_WAIT(cs_bar, read_barrier());
        }
        }
        if (++cc == nchunk) {
            // (explicit calls: a loop around the inlined epilogue cost the allocator ~240
            // spilled registers)
            if constexpr (PAIR) {
                // (host: bf16-only output, no accumulate, no BatchNorm-backward partials, W % 32
                // == 0) both n-tiles as whole lines; only this epilogue is compiled in
                static_assert(NP == 1 && NT == 2 && TW == 32, "the 4 x 2-tile single-piece forms");
                if constexpr (PAIR == 2)  // (host: with BN-backward partials of a bf16 y)
                    CS_WAIT(cs_epi, (x6_epilogue_pair16_bnb<TH, TW, MT, WM>(
                                        a, acc[0], acc[1], cp.tile, cp.b, cp.ty0, cp.tx0,
                                        cp.nb * BNI + wn * NT * 32, wm, ostg + wave * NT * X6_STG_WAVE)));
                else
                    CS_WAIT(cs_epi, (x6_epilogue_pair16<TH, TW, MT, WM>(
                                        a, acc[0], acc[1], cp.tile, cp.b, cp.ty0, cp.tx0,
                                        cp.nb * BNI + wn * NT * 32, wm, ostg + wave * NT * X6_STG_WAVE)));
            } else if constexpr (TW == 16) {
                // 16-wide image (host: W == 16, H even): a 32-pixel m-tile is two whole image
                // rows, so the NHWC addresses are those of a 32-wide image of half the rows --
                // the 32-wide epilogue on that view, every tile full width
                static_assert(NT == 1, "one n-tile per wave");
                ConvFwdArgs av = a;
                av.H = a.H / 2;
                av.W = 32;
                CS_WAIT(cs_epi, (x6_epilogue_wave<TH / 2, 32, MT, WM, true, true>(
                                    av, acc[0], cp.tile, cp.b, cp.ty0 / 2, 0, cp.nb * BNI + wn * 32,
                                    wm, ostg + wave * X6_STG_WAVE)));
            } else
#ifdef X6R_NO_FW  // A/B build: the per-pixel column guards everywhere
            if (false) {
#else
            if (cp.tx0 + TW <= a.W) {  // (uniform) the common case: a full-width tile
#endif
                CS_WAIT(cs_epi, (x6_epilogue_wave<TH, TW, MT, WM, NT == 1, true>(
                                    a, acc[0], cp.tile, cp.b, cp.ty0, cp.tx0, cp.nb * BNI + wn * NT * 32,
                                    wm, ostg + wave * NT * X6_STG_WAVE)));
                if constexpr (NT > 1)
                    CS_WAIT(cs_epi, (x6_epilogue_wave<TH, TW, MT, WM, NT == 1, true>(
                                        a, acc[1], cp.tile, cp.b, cp.ty0, cp.tx0,
                                        cp.nb * BNI + (wn * NT + 1) * 32, wm,
                                        ostg + (wave * NT + 1) * X6_STG_WAVE)));
            } else {
                CS_WAIT(cs_epi, (x6_epilogue_wave<TH, TW, MT, WM, NT == 1>(
                                    a, acc[0], cp.tile, cp.b, cp.ty0, cp.tx0, cp.nb * BNI + wn * NT * 32,
                                    wm, ostg + wave * NT * X6_STG_WAVE)));
                if constexpr (NT > 1)
                    CS_WAIT(cs_epi, (x6_epilogue_wave<TH, TW, MT, WM, NT == 1>(
                                        a, acc[1], cp.tile, cp.b, cp.ty0, cp.tx0,
                                        cp.nb * BNI + (wn * NT + 1) * 32, wm,
                                        ostg + (wave * NT + 1) * X6_STG_WAVE)));
            }
            static_assert(NT <= 2, "two n-tiles at most");
            if constexpr (NP == 1 && NT > 1) {
                // the next step's first taps, not held in registers across the epilogue
#pragma unroll
                for (int t = 0; t < PD; ++t) ldfrag1(k + 1, t, fa1[t], fb1[t]);
            }
            cc = 0;
            item += nslots;
            if (item < iend) cp = pos_of(item);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[nt][mt][r] = 0.f;
        }
    }
#ifdef X6R_CLOCK
    if (tid == 0 && blockIdx.x < 4096) {
        g_clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - clk_t0;
        g_clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - clk_r0;
    }
#endif
    CS_STORE();
    }
#undef CS_WAIT
#undef CS_STORE
}
// ---------------------------------------------------------------------------
// Split-bf16 weight gradient: dW[co][ci][t] = sum_p dy[p][co] * act(x)[p+t][ci].
// Same item decomposition and partial layout as conv3x3_wgrad_kernel (64 co x
// 64 ci x 9 taps per item, 4 compute waves as 2 (co) x 2 (ci) with nine 32x32
// accumulators, deterministic split-K), but the K = pixel reduction runs on
// v_mfma_f32_32x32x16_bf16: one k-step = one 16-pixel row of the 4 x 16 tile.
// Both operands are pixel-major in LDS -- one 448-B record per pixel holding the
// three bf16 pieces of its 64 channels (384 B + 64 B pad) -- and are read
// transposed with ds_read_b64_tr_b16 (4 pixels x 16 channels per 16-lane group):
// the tap shift is then just a constant record offset, and the 112-dword record
// pitch puts any 4 consecutive pixels x 32 channels on 64 distinct banks.
// ---------------------------------------------------------------------------
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3_4(f32x4 v, u32x2& p0, u32x2& p1, u32x2& p2) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        unsigned a, b, c;
        split3_pair(v[2 * i], v[2 * i + 1], a, b, c);
        p0[i] = a;
        p1[i] = b;
        p2[i] = c;
    }
}

template <int NP>
__device__ __forceinline__ void split_n4(f32x4 v, u32x2 (&p)[NP]) {
    if constexpr (NP == 3) {
        split3_4(v, p[0], p[1], p[2]);
    } else {
        p[0] = __builtin_bit_cast(u32x2, __builtin_convertvector(v, bf16x4));
    }
}

__device__ __forceinline__ u32x2 ds_read_tr(const char* lds_byte_addr) {
    const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(lds_byte_addr));
    return __builtin_bit_cast(u32x2, v);
}

constexpr int WX_REC = 448;  // bytes per pixel record: 3 pieces x 64 ch x 2 B + 64 B pad

// ---------------------------------------------------------------------------
// Persistent, warp-specialized form of the split-bf16 weight gradient ("x6w"),
// one 8-wave workgroup per CU walking a contiguous
// per-XCD range of items (64-co block, 64-ci block, pixel split); waves 0-3 only
// read fragments and issue MFMAs, waves 4-7 stage: during step k (one 2 x 16
// pixel tile) they write tile k+1 into the idle half of a double-buffered LDS
// image from registers loaded during step k-1, then issue the loads of tile k+2
// (untracked loads + counted vmcnt, so they stay in flight across the barrier).
// ---------------------------------------------------------------------------
// record pitch of the wgrad LDS images: NP pieces x 64 ch x 2 B, padded so that 4
// consecutive records x 32 channels cover 64 distinct banks (pitch = 48 dwords mod 64)
template <int NP>
constexpr int wrec() { return NP == 3 ? WX_REC : 192; }

// (A paired 16x16x32 form, as the forward's, measured 2 % slower: 32x32x16 it is.)
// XB bit 1: the activation operand is stored in bf16 (a.src*_16), bit 2: dy is (a.dy16) --
// the bf16 arithmetic's storage, NP = 1: 8-byte loads of 4 channels instead of 16-byte
// ones, same load count per step
// BN: dy is formed while loading from the following BatchNorm(+ReLU) backward (a.bn_*:
// da, y and the apply's coefficients; bn_bwd_dy, bit-identical to the apply pass) and, by
// the items of the first input-channel block, written to a.bn_dy_out for the data gradient
// -- the BatchNorm-backward apply pass folded into the loader waves, which wait at
// barriers 15-29 % of the loop in this form (profiles/r4n_x6w_stamps_x6.txt)
template <int TH, int TW, int NP, int XB = 0, bool BN = false>
__global__ void __launch_bounds__(512, 1) conv3x3_wgrad_x6w_kernel(WgradArgs a) {
    constexpr bool XB16 = (XB & 1) != 0, DB16 = (XB & 2) != 0;
    static_assert(XB == 0 || NP == 1, "bf16 storage: single-piece arithmetic");
    // (BN in the single-piece form: its loaders already wait on loads 11-22 % of the loop,
    // and folding the apply there made the bf16 step 1.6 % slower, profiles/r5j_*)
    static_assert(!BN || (NP == 3 && XB == 0), "lazy BatchNorm-backward dy: split-bf16 form");
    constexpr int REC = wrec<NP>();
    static_assert(TW == 16, "one 16-pixel row per MFMA k-step");
    constexpr int P = TH * TW, HWD = TW + 2, NHALO = (TH + 2) * HWD;
    constexpr int DY_Q = P * 16, X_Q = NHALO * 16;  // float4 quads per tile
    constexpr int DY_PER = (DY_Q + 255) / 256, X_PER = (X_Q + 255) / 256;
    constexpr int RECS = P + NHALO;                  // records per buffer
    // loader untracked VMEM per step: dY, X, the two coefficient loads and, with the lazy
    // BatchNorm-backward dy, the y loads plus the max-pool route's pooled-gradient and argmax
    // loads (2 * DY_PER, an upper bound: issued only on routed launches).  Only counted waits
    // of earlier register sets use it (NSET > 1), which BN excludes today (static_assert below)
    // O8: bf16 dy and activations (XB == 3, the bf16 arithmetic's weight gradient): 16-byte
    // loads of 8 channels, 8 lanes per pixel -- 2 + 4 loads per step for the 64-pixel tile and
    // its halo instead of 4 + 7 of 4 channels (the loaders spend 41-57 % of this form's loop
    // issuing loads: profiles/r7c_ab_x6w_o8.txt) -- and 16-byte LDS record stores
#ifndef X6W_O8  // (A/B build: -D X6W_O8=0, 8-byte loads of 4 channels)
#define X6W_O8 1
#endif
    constexpr bool O8 = X6W_O8 && NP == 1 && XB16 && DB16 && !BN;
    constexpr int DY_PER8 = (P * 8 + 255) / 256, X_O8 = NHALO * 8, X_PER8 = (X_O8 + 255) / 256;
    static_assert(P * 8 % 256 == 0, "whole dy rounds");
    constexpr int LOADS = O8 ? DY_PER8 + X_PER8 + 4 : DY_PER + X_PER + 2 + (BN ? 3 * DY_PER : 0);
    __shared__ __attribute__((aligned(16))) char smem[(2 * RECS + 1) * REC];
    char* const dummy = smem + 2 * RECS * REC;    // record for idle lanes' writes

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool loader = wave >= 4;
    const int NCO = a.Cout / 64, NCI = a.Cin / 64;
    const int nitems = NCO * NCI * a.nsplit;
    const int nslots = gridDim.x >> 3;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int iq = nitems >> 3, ir = nitems & 7;
    const int ibeg = xcd * iq + min(xcd, ir);
    const int iend = ibeg + iq + (xcd < ir ? 1 : 0);
    const int item0 = ibeg + slot;
    if (item0 >= iend) return;  // uniform per workgroup
    const int tpi = a.tiles_x * a.tiles_y;

    // flat step sequence: the tiles of item0, then of item0 + nslots, ...
    struct Cur {
        int item, tile, tend;
    };
    auto item_range = [&](int it, Cur& c) {
        const int split = it / (NCO * NCI);
        c.item = it;
        c.tile = split * a.tps;
        c.tend = min(a.ntiles, c.tile + a.tps);
    };
    auto advance = [&](Cur& c) {  // stays on the last step past the end
        if (c.tile + 1 < c.tend) {
            ++c.tile;
        } else if (c.item + nslots < iend) {
            item_range(c.item + nslots, c);
        }
    };
    int total = 0;
    for (int it = item0; it < iend; it += nslots) {
        Cur c;
        item_range(it, c);
        total += max(c.tend - c.tile, 0);
    }
    if (total == 0) return;

    if (loader) {
        // ------------------------------------------------------------ loader waves
        const int lt = tid - 256;
        // NSET register sets: the single-piece form (NP = 1) keeps two steps' loads in
        // flight (its steps are a third as long, and one step of flight left the loaders
        // waiting 11-22 % of the loop in vmcnt: tools/clock_probe.py --stamps --wgrad)
#ifndef X6W_NSET1  // (A/B builds: 3 sets measured neutral, profiles/r5l_ab_x6w_three_sets_bf16.txt)
#define X6W_NSET1 2
#endif
        constexpr int NSET = NP == 1 ? X6W_NSET1 : 1;
        typename std::conditional<DB16, u32x2v, f32x4>::type rdy[NSET][DY_PER];
        typename std::conditional<XB16, u32x2v, f32x4>::type rx[NSET][X_PER];
        Act4 xa[NSET];
        float xlo[NSET];
        unsigned dvalid[NSET], xvalid[NSET];
        // BN: y beside da, the lane's 4 channels' (scale, shift, mean, invstd, k0, k1), and
        // where (and whether: first ci block) the formed dy goes
        f32x4 rby[BN ? NSET : 1][BN ? DY_PER : 1], bco[BN ? NSET : 1][6];
        // BN with a MaxPool2d route: the pooled gradient and argmax bytes of each vector's
        // pixel, and the pixel's window position (255: outside the pooled area)
        f32x4 rrs[BN ? NSET : 1][BN ? DY_PER : 1];
        unsigned ram[BN ? NSET : 1][BN ? DY_PER : 1], rkk[BN ? NSET : 1][BN ? DY_PER : 1];
        int bco_nb = -1;  // output-channel block whose coefficients bco holds
        static_assert(!BN || NSET == 1, "one coefficient set");
        bool bwr[NSET];
        size_t bbase[NSET];
        int bof[BN ? NSET : 1][BN ? DY_PER : 1];
        // the loader's cursor also carries the item's co / ci blocks and the tile's
        // image position, updated without divisions inside an item
        struct LCur {
            Cur c;
            int nb, cb, b, ty0, tx0;
        };
        auto lderive = [&](LCur& l) {
            l.nb = l.c.item % NCO;
            l.cb = (l.c.item / NCO) % NCI;
            const int trem = l.c.tile % tpi;
            l.b = l.c.tile / tpi;
            l.ty0 = (trem / a.tiles_x) * TH;
            l.tx0 = (trem % a.tiles_x) * TW;
        };
        auto ladvance = [&](LCur& l) {  // stays on the last step past the end
            if (l.c.tile + 1 < l.c.tend) {
                ++l.c.tile;
                l.tx0 += TW;
                if (l.tx0 >= a.tiles_x * TW) {
                    l.tx0 = 0;
                    l.ty0 += TH;
                    if (l.ty0 >= a.tiles_y * TH) {
                        l.ty0 = 0;
                        ++l.b;
                    }
                }
            } else if (l.c.item + nslots < iend) {
                item_range(l.c.item + nslots, l.c);
                lderive(l);
            }
        };
        // the lane's element offsets from the tile origin for interior tiles (every dy and
        // halo pixel inside the image): step-invariant, computed once (one set per source,
        // whose channel counts differ) instead of two integer multiplies per vector per step
        int dof_in[DY_PER], xof_in[2][X_PER];
        unsigned xin_all = 0;
#pragma unroll
        for (int v = 0; v < DY_PER; ++v) {
            const int p = (lt + v * 256) >> 4;
            dof_in[v] = ((p / TW) * a.W + p % TW) * a.Cout;
        }
#pragma unroll
        for (int v = 0; v < X_PER; ++v) {
            const int idx = lt + v * 256;
            const int hp = idx < X_Q ? idx >> 4 : 0;
            const int o = (hp / HWD - 1) * a.W + hp % HWD - 1;
            xof_in[0][v] = idx < X_Q ? o * a.C0 : 0;
            xof_in[1][v] = idx < X_Q ? o * a.C1 : 0;
            xin_all |= (idx < X_Q ? 1u : 0u) << v;
        }
        // O8 state: 8 bf16 per vector, the lane's 8 channels' activation coefficients
        f32x4 rdy8[O8 ? NSET : 1][O8 ? DY_PER8 : 1], rx8[O8 ? NSET : 1][O8 ? X_PER8 : 1];
        Act4 xa8[O8 ? NSET : 1][2];
        int dof8_in[O8 ? DY_PER8 : 1], xof8_in[2][O8 ? X_PER8 : 1];
        unsigned xin8_all = 0;
        if constexpr (O8) {
#pragma unroll
            for (int v = 0; v < DY_PER8; ++v) {
                const int p = (lt + v * 256) >> 3;
                dof8_in[v] = ((p / TW) * a.W + p % TW) * a.Cout;
            }
#pragma unroll
            for (int v = 0; v < X_PER8; ++v) {
                const int idx = lt + v * 256;
                const int hp = idx < X_O8 ? idx >> 3 : 0;
                const int o = (hp / HWD - 1) * a.W + hp % HWD - 1;
                xof8_in[0][v] = idx < X_O8 ? o * a.C0 : 0;
                xof8_in[1][v] = idx < X_O8 ? o * a.C1 : 0;
                xin8_all |= (idx < X_O8 ? 1u : 0u) << v;
            }
        }
        auto gload8 = [&](const LCur& c, auto S) {
            constexpr int st = decltype(S)::value;
            const int co0 = c.nb * 64, ci0 = c.cb * 64;
            const bool second = ci0 >= a.C0;
            const __bf16* xsrc16 = second ? a.src1_16 : a.src0_16;
            const float* xsc = second ? a.sc1 : a.sc0;
            const float* xsh = second ? a.sh1 : a.sh0;
            const int Cs = second ? a.C1 : a.C0, cbase = second ? ci0 - a.C0 : ci0;
            const bool xon = xsc != nullptr;
            xlo[st] = xon ? 0.f : -INFINITY;
            const int o8 = (lt & 7) * 8;
            const float* scp = (xon ? xsc : g_act_ones) + cbase + o8;
            const float* shp = (xon ? xsh : g_act_zeros) + cbase + o8;
            xa8[st][0].s = gld16(scp);
            xa8[st][0].h = gld16(shp);
            xa8[st][1].s = gld16(scp + 4);
            xa8[st][1].h = gld16(shp + 4);
            const int b = c.b, ty0 = c.ty0, tx0 = c.tx0;
            int dof[DY_PER8], xof[X_PER8];
            if (ty0 >= 1 && tx0 >= 1 && ty0 + TH + 1 <= a.H && tx0 + TW + 1 <= a.W) {
                // interior tile (uniform): every dy pixel and halo pixel is in the image
#pragma unroll
                for (int v = 0; v < DY_PER8; ++v) dof[v] = dof8_in[v];
#pragma unroll
                for (int v = 0; v < X_PER8; ++v) xof[v] = second ? xof8_in[1][v] : xof8_in[0][v];
                dvalid[st] = (1u << DY_PER8) - 1;
                xvalid[st] = xin8_all;
            } else {
                dvalid[st] = 0;
#pragma unroll
                for (int v = 0; v < DY_PER8; ++v) {
                    const int p = (lt + v * 256) >> 3;
                    const int gy = ty0 + p / TW, gx = tx0 + p % TW;
                    const bool ok = gy < a.H && gx < a.W;
                    const int cy = min(gy, a.H - 1), cx = min(gx, a.W - 1);
                    dof[v] = ((cy - ty0) * a.W + (cx - tx0)) * a.Cout;
                    dvalid[st] |= (ok ? 1u : 0u) << v;
                }
                xvalid[st] = 0;
#pragma unroll
                for (int v = 0; v < X_PER8; ++v) {
                    const int idx = lt + v * 256;
                    const int hp = idx < X_O8 ? idx >> 3 : 0;
                    const int gy = ty0 + hp / HWD - 1, gx = tx0 + hp % HWD - 1;
                    const bool ok = idx < X_O8 && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W;
                    const int cy = min(max(gy, 0), a.H - 1), cx = min(max(gx, 0), a.W - 1);
                    xof[v] = ((cy - ty0) * a.W + (cx - tx0)) * Cs;
                    xvalid[st] |= (ok ? 1u : 0u) << v;
                }
            }
            const size_t dyo0 = ((size_t)(b * a.H + ty0) * a.W + tx0) * a.Cout + co0 + o8;
            const size_t xb = ((size_t)(b * a.H + ty0) * a.W + tx0) * Cs + cbase + o8;
#pragma unroll
            for (int v = 0; v < DY_PER8; ++v) rdy8[st][v] = gld16(a.dy16 + dyo0 + dof[v]);
#pragma unroll
            for (int v = 0; v < X_PER8; ++v) rx8[st][v] = gld16(xsrc16 + xb + xof[v]);
        };
        auto gload = [&](const LCur& c, auto S) {
            if constexpr (O8) {
                gload8(c, S);
                return;
            }
            constexpr int st = decltype(S)::value;
            const int co0 = c.nb * 64, ci0 = c.cb * 64;
            const bool second = ci0 >= a.C0;
            const float* xsrc = second ? a.src1 : a.src0;
            const __bf16* xsrc16 = second ? a.src1_16 : a.src0_16;
            const float* xsc = second ? a.sc1 : a.sc0;
            const float* xsh = second ? a.sh1 : a.sh0;
            const int Cs = second ? a.C1 : a.C0, cbase = second ? ci0 - a.C0 : ci0;
            const bool xon = xsc != nullptr;
            xlo[st] = xon ? 0.f : -INFINITY;
            const int cq = cbase + (lt & 15) * 4;  // q = idx & 15 = lt & 15
            xa[st].s = gld16((xon ? xsc : g_act_ones) + cq);
            xa[st].h = gld16((xon ? xsh : g_act_zeros) + cq);
            const int b = c.b, ty0 = c.ty0, tx0 = c.tx0;
            const int q4 = (lt & 15) * 4;
            // per-lane pixel positions inside the tile (compile-time divisors): dy
            // pixels, and halo pixels relative to the tile origin (-1, -1)
            int dyo[DY_PER], xpy[X_PER], xpx[X_PER];
            unsigned xin = 0;  // x vectors that exist (idx < X_Q)
#pragma unroll
            for (int v = 0; v < DY_PER; ++v) {
                const int p = (lt + v * 256) >> 4;
                dyo[v] = (p / TW) * a.W + p % TW;
            }
#pragma unroll
            for (int v = 0; v < X_PER; ++v) {
                const int idx = lt + v * 256;
                const int hp = idx < X_Q ? idx >> 4 : 0;
                xpy[v] = hp / HWD - 1;
                xpx[v] = hp % HWD - 1;
                xin |= (idx < X_Q ? 1u : 0u) << v;
            }
            // element offsets from the tile origin; only integer work depends on whether
            // the tile touches the image border, the loads are one straight sequence
            // (a load inside a branch would leave its registers in flight on the
            // structurized path that skips it)
            int dof[DY_PER], xof[X_PER];
            if (ty0 >= 1 && tx0 >= 1 && ty0 + TH + 1 <= a.H && tx0 + TW + 1 <= a.W) {
                // interior tile (uniform): every dy pixel and halo pixel is in the image
#pragma unroll
                for (int v = 0; v < DY_PER; ++v) dof[v] = dof_in[v];
#pragma unroll
                for (int v = 0; v < X_PER; ++v) xof[v] = second ? xof_in[1][v] : xof_in[0][v];
                dvalid[st] = (1u << DY_PER) - 1;
                xvalid[st] = xin_all;
            } else {
                dvalid[st] = 0;
#pragma unroll
                for (int v = 0; v < DY_PER; ++v) {
                    const int p = (lt + v * 256) >> 4;
                    const int gy = ty0 + p / TW, gx = tx0 + p % TW;
                    const bool ok = gy < a.H && gx < a.W;
                    const int cy = min(gy, a.H - 1), cx = min(gx, a.W - 1);
                    dof[v] = ((cy - ty0) * a.W + (cx - tx0)) * a.Cout;
                    dvalid[st] |= (ok ? 1u : 0u) << v;
                }
                xvalid[st] = 0;
#pragma unroll
                for (int v = 0; v < X_PER; ++v) {
                    const int gy = ty0 + xpy[v], gx = tx0 + xpx[v];
                    const bool ok =
                        ((xin >> v) & 1u) && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W;
                    const int cy = min(max(gy, 0), a.H - 1), cx = min(max(gx, 0), a.W - 1);
                    xof[v] = ((cy - ty0) * a.W + (cx - tx0)) * Cs;
                    xvalid[st] |= (ok ? 1u : 0u) << v;
                }
            }
            const size_t dyo0 = ((size_t)(b * a.H + ty0) * a.W + tx0) * a.Cout + co0 + q4;
            const size_t xb = ((size_t)(b * a.H + ty0) * a.W + tx0) * Cs + cbase + q4;
            if constexpr (BN) {
                // the lane's coefficients change with the output-channel block only: plain
                // (tracked) loads at an item's first step (NSET = 1: consumed by this set)
#ifndef X6W_BN_COEF_PER_STEP
                if (c.nb != bco_nb)
#endif
                {
                    bco_nb = c.nb;
                    const int cq = co0 + q4;
                    auto ld = [](const float* q) { return *reinterpret_cast<const f32x4*>(q); };
                    bco[st][0] = ld(a.bn_scale + cq);
                    bco[st][1] = ld(a.bn_shift + cq);
                    bco[st][2] = ld(a.bn_mean + cq);
                    bco[st][3] = ld(a.bn_invstd + cq);
                    bco[st][4] = ld(a.bn_coef + cq);
                    bco[st][5] = ld(a.bn_coef + a.Cout + cq);
                }
                bwr[st] = a.bn_dy_out != nullptr && c.cb == 0;
                bbase[st] = dyo0;
            }
#pragma unroll
            for (int v = 0; v < DY_PER; ++v) {
                if constexpr (BN) {
                    // (no base gradient with a route: y's address stands in, the value unused --
                    // the loads stay one straight sequence)
                    rdy[st][v] = gld16((a.bn_da ? a.bn_da : a.bn_y) + dyo0 + dof[v]);
                    rby[st][v] = gld16(a.bn_y + dyo0 + dof[v]);
                    bof[st][v] = dof[v];
                    if (a.bn_rsrc) {  // (uniform)
                        const int p = (lt + v * 256) >> 4;
                        const int gy = ty0 + p / TW, gx = tx0 + p % TW, Ho = a.H >> 1, Wo = a.W >> 1;
                        const bool rok = gy < a.H && gx < a.W && (gy >> 1) < Ho && (gx >> 1) < Wo;
                        const size_t ro = (rok ? ((size_t)(b * Ho + (gy >> 1)) * Wo + (gx >> 1)) * a.Cout : 0) +
                                          co0 + q4;
                        rrs[st][v] = gld16(a.bn_rsrc + ro);
                        ram[st][v] = gld4(a.bn_ram + ro);
                        rkk[st][v] = rok ? (unsigned)((gy & 1) * 2 + (gx & 1)) : 255u;
                    }
                } else if constexpr (DB16) {
                    rdy[st][v] = gld8(a.dy16 + dyo0 + dof[v]);
                } else {
                    rdy[st][v] = gld16(a.dy + dyo0 + dof[v]);
                }
            }
#pragma unroll
            for (int v = 0; v < X_PER; ++v) {
                if constexpr (XB16) rx[st][v] = gld8(xsrc16 + xb + xof[v]);
                else rx[st][v] = gld16(xsrc + xb + xof[v]);
            }
        };
        // record layout: [piece][64 ch] bf16 at byte piece*128 + ch*2
        auto put = [&](char* rec, int q, f32x4 v) {
            u32x2 pc[NP];
            split_n4<NP>(v, pc);
            char* r = rec + q * 8;
#pragma unroll
            for (int k = 0; k < NP; ++k) *reinterpret_cast<u32x2*>(r + 128 * k) = pc[k];
        };
        auto lstore8 = [&](int buf, auto S) {
            constexpr int st = decltype(S)::value;
            char* dys = smem + buf * RECS * REC;
            char* xs = dys + P * REC;
            // record layout [64 ch] bf16: lane (pixel, o) writes channels 8o..8o+7 (16 B; an
            // 8-lane store group covers one pixel's 128 contiguous bytes: conflict-free)
#pragma unroll
            for (int v = 0; v < DY_PER8; ++v) {
                const int idx = lt + v * 256;
                const bool ok = (dvalid[st] >> v) & 1u;
                u32x4 w = __builtin_bit_cast(u32x4, rdy8[st][v]);
#pragma unroll
                for (int i = 0; i < 4; ++i) w[i] = ok ? w[i] : 0u;
                *reinterpret_cast<u32x4*>(dys + (idx >> 3) * REC + (idx & 7) * 16) = w;
            }
            const bool act = xlo[st] > -INFINITY;  // (uniform) else the bits as they are
#pragma unroll
            for (int v = 0; v < X_PER8; ++v) {
                const int idx = lt + v * 256;
                const bool ok = (xvalid[st] >> v) & 1u;
                u32x4 w = __builtin_bit_cast(u32x4, rx8[st][v]);
                if (act) {
                    f32x4 lo4, hi4;  // 8 bf16 widened (exact), activated, rounded back
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        lo4[2 * i] = __uint_as_float(w[i] << 16);
                        lo4[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
                        hi4[2 * i] = __uint_as_float(w[2 + i] << 16);
                        hi4[2 * i + 1] = __uint_as_float(w[2 + i] & 0xffff0000u);
                    }
                    lo4 = act_floor4(lo4, xa8[st][0], xlo[st]);
                    hi4 = act_floor4(hi4, xa8[st][1], xlo[st]);
                    u32x2 pl[1], ph[1];
                    split_n4<1>(lo4, pl);
                    split_n4<1>(hi4, ph);
                    w = u32x4{pl[0].x, pl[0].y, ph[0].x, ph[0].y};
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) w[i] = ok ? w[i] : 0u;
                *reinterpret_cast<u32x4*>((idx < X_O8 ? xs + (idx >> 3) * REC : dummy) + (idx & 7) * 16) = w;
            }
        };
        auto lstore = [&](int buf, auto S) {
            if constexpr (O8) {
                lstore8(buf, S);
                return;
            }
            constexpr int st = decltype(S)::value;
            char* dys = smem + buf * RECS * REC;
            char* xs = dys + P * REC;
#pragma unroll
            for (int v = 0; v < DY_PER; ++v) {
                const int idx = lt + v * 256;
                if constexpr (NP == 1 && DB16 && !BN) {
                    // bf16 dy is already the single piece: its bits go to the record as they
                    // are (the widen / round trip through fp32 was exact and cost 10 VALU)
                    const bool ok = (dvalid[st] >> v) & 1u;
                    const u32x2 w = {ok ? rdy[st][v].x : 0u, ok ? rdy[st][v].y : 0u};
                    *reinterpret_cast<u32x2*>(dys + (idx >> 4) * REC + (idx & 15) * 8) = w;
                    continue;
                }
                const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                f32x4 d;
                if constexpr (DB16)  // 4 bf16 widened (exact)
                    d = f32x4{__uint_as_float(rdy[st][v].x << 16), __uint_as_float(rdy[st][v].x & 0xffff0000u),
                              __uint_as_float(rdy[st][v].y << 16), __uint_as_float(rdy[st][v].y & 0xffff0000u)};
                else
                    d = rdy[st][v];
                const bool ok = (dvalid[st] >> v) & 1u;
                if constexpr (BN) {
                    if (a.bn_rsrc) {  // (uniform) da = routed + base, in the apply's order
                        f32x4 g;
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            g[i] = ((ram[st][v] >> (8 * i)) & 0xffu) == rkk[st][v] ? rrs[st][v][i] : 0.f;
                        if (a.bn_da) {
#pragma unroll
                            for (int i = 0; i < 4; ++i) g[i] += d[i];
                        }
                        d = g;
                    }
                    const f32x4 yv = rby[st][v];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        d[i] = bn_bwd_dy(d[i], yv[i], bco[st][0][i], bco[st][1][i], bco[st][2][i],
                                         bco[st][3][i], bco[st][4][i], bco[st][5][i]);
                    if (bwr[st] && ok)  // (uniform bwr: one store per vector, then the next)
                        *reinterpret_cast<f32x4*>(a.bn_dy_out + bbase[st] + bof[st][v]) = d;
                }
                put(dys + (idx >> 4) * REC, idx & 15, ok ? d : z);
            }
            if constexpr (NP == 1 && XB16) {
                if (!(xlo[st] > -INFINITY)) {  // (uniform) no activation: the bits as they are
#pragma unroll
                    for (int v = 0; v < X_PER; ++v) {
                        const int idx = lt + v * 256;
                        const bool ok = (xvalid[st] >> v) & 1u;
                        const u32x2 w = {ok ? rx[st][v].x : 0u, ok ? rx[st][v].y : 0u};
                        *reinterpret_cast<u32x2*>((idx < X_Q ? xs + (idx >> 4) * REC : dummy) +
                                                  (idx & 15) * 8) = w;
                    }
                    return;
                }
            }
#pragma unroll
            for (int v = 0; v < X_PER; ++v) {
                const int idx = lt + v * 256;
                const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                f32x4 raw;
                if constexpr (XB16)  // 4 bf16 widened (exact)
                    raw = f32x4{__uint_as_float(rx[st][v].x << 16), __uint_as_float(rx[st][v].x & 0xffff0000u),
                                __uint_as_float(rx[st][v].y << 16), __uint_as_float(rx[st][v].y & 0xffff0000u)};
                else
                    raw = rx[st][v];
                const f32x4 val = ((xvalid[st] >> v) & 1u) ? act_floor4(raw, xa[st], xlo[st]) : z;
                put(idx < X_Q ? xs + (idx >> 4) * REC : dummy, idx & 15, val);
            }
        };
        using Set0 = std::integral_constant<int, 0>;
        // step s's loads go to register set s % NSET
        LCur lc;
        item_range(item0, lc.c);
        lderive(lc);
        gload(lc, Set0{});
        vm_wait<0>();
        lstore(0, Set0{});
        ladvance(lc);
        gload(lc, std::integral_constant<int, 1 % NSET>{});  // step 1
        if constexpr (NSET >= 2) {
            ladvance(lc);
            gload(lc, std::integral_constant<int, 2 % NSET>{});  // step 2
        }
        if constexpr (NSET >= 3) {
            ladvance(lc);
            gload(lc, Set0{});  // step 3 (set 0 was stored above)
        }
        static_assert(NSET <= 3, "at most three register sets");
        lds_barrier();
#ifdef X6W_STAMP
        // diagnostic build: loader cycles waiting for global loads / at the barrier
        unsigned long long st_vm = 0, st_bar = 0, st_ls = 0, st_gl = 0;  // + LDS stores, loads
        const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
#define ST_WAIT(acc, stmt)                                          \
    {                                                               \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        stmt;                                                       \
        acc += __builtin_amdgcn_s_memtime() - t_;                   \
    }
#else
#define ST_WAIT(acc, stmt) stmt
#endif
        // step k: write step k+1 (its loads retired: with two sets, step k+2's stay in
        // flight -- loads retire in issue order), then issue step k+1+NSET into the freed set
        auto lstep = [&](int k, auto S) {
            if constexpr (NSET >= 2) {  // steps k+2 .. k+NSET stay in flight
                ST_WAIT(st_vm, vm_wait<(NSET - 1) * LOADS>());
            } else {
                ST_WAIT(st_vm, vm_wait<0>());
            }
            ST_WAIT(st_ls, lstore((k + 1) & 1, S));  // step k+1
            ST_WAIT(st_gl, ladvance(lc); gload(lc, S));  // step k+1+NSET, in flight across the barrier
            ST_WAIT(st_bar, lds_barrier());
        };
        for (int k = 0; k < total; k += NSET) {  // lstep(k) stores step k+1: set (k+1) % NSET
            lstep(k, std::integral_constant<int, 1 % NSET>{});
            if constexpr (NSET >= 2)
                if (k + 1 < total) lstep(k + 1, std::integral_constant<int, 2 % NSET>{});
            if constexpr (NSET >= 3)
                if (k + 2 < total) lstep(k + 2, Set0{});
        }
#undef ST_WAIT
        vm_wait<0>();  // no load outlives the workgroup (nothing may run before this wait:
                       // the last loads' destination registers are dead to the compiler)
#ifdef X6W_STAMP
        if (tid == 256 && blockIdx.x < 512) {
            g_clk[16 * blockIdx.x] = __builtin_amdgcn_s_memtime() - st_t0;
            g_clk[16 * blockIdx.x + 1] = st_vm;
            g_clk[16 * blockIdx.x + 4] = st_bar;
            g_clk[16 * blockIdx.x + 12] = st_ls;
            g_clk[16 * blockIdx.x + 13] = st_gl;
        }
#endif
        return;
    }

    // ---------------------------------------------------------------- compute waves
    const int wm = wave >> 1, wn = wave & 1;
    f32x16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    // transposed-read addresses: 16-lane group g = lane>>4 (h = g>>1 pixel half,
    // g&1 channel half), lane li supplies row (pixel) li>>2, channels 4(li&3)..+3.
    const int li = lane & 15, g = lane >> 4, hh = g >> 1;
    const int pix_in = 8 * hh + (li >> 2);
    const int ch_a = wm * 32 + 16 * (g & 1) + 4 * (li & 3);
    const int ch_b = wn * 32 + 16 * (g & 1) + 4 * (li & 3);
    Cur cc;
    item_range(item0, cc);
    lds_barrier();  // step 0 staged
    for (int k = 0; k < total; ++k) {
        const char* dys = smem + (k & 1) * RECS * REC;
        const char* abase = dys + pix_in * REC + ch_a * 2;
        const char* bbase = dys + P * REC + pix_in * REC + ch_b * 2;
        auto lda = [&](int ks, u32x4 (&af)[NP]) {
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const char* pa = abase + ks * TW * REC + q * 128;
                const u32x2 lo = ds_read_tr(pa), hi = ds_read_tr(pa + 4 * REC);
                af[q] = u32x4{lo.x, lo.y, hi.x, hi.y};
            }
        };
        auto ldb = [&](int ks, int t, u32x4 (&bf)[NP]) {
            const char* pb = bbase + ((ks + t / 3) * HWD + (t % 3)) * REC;
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const u32x2 lo = ds_read_tr(pb + q * 128), hi = ds_read_tr(pb + q * 128 + 4 * REC);
                bf[q] = u32x4{lo.x, lo.y, hi.x, hi.y};
            }
        };
        // TH rows x 9 taps as one sequence: the fragments of unit u + BD (a tap; and the
        // dy fragments of the next row) are read during unit u's MFMAs
#ifndef X6W_BDEPTH3  // (A/B builds: read depth in units, split-bf16 / single-piece forms)
#define X6W_BDEPTH3 1
#endif
#ifndef X6W_BDEPTH1
#define X6W_BDEPTH1 1
#endif
        constexpr int BD = NP == 3 ? X6W_BDEPTH3 : X6W_BDEPTH1, NU = 9 * TH;
        static_assert(BD >= 1 && BD <= 8, "read depth");
        u32x4 afr[2][NP], bfr[BD + 1][NP];
#pragma unroll
        for (int v = 0; v < BD; ++v) {
            if (v % 9 == 0) lda(v / 9, afr[(v / 9) & 1]);
            ldb(v / 9, v % 9, bfr[v]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int ks = u / 9, t = u % 9, un = u + BD;
            // (row un/9's dy fragments go to the buffer row un/9 - 2 used: done, BD <= 8)
            if (un < NU) {
                if (un % 9 == 0) lda(un / 9, afr[(un / 9) & 1]);
                ldb(un / 9, un % 9, bfr[un % (BD + 1)]);
            }
            acc[t] = mfma_xn<NP>(afr[ks & 1], bfr[u % (BD + 1)], acc[t]);
            // next fragments (2 reads per piece, twice that at a row change) spread over
            // the first half of the tap's MFMA gaps
            const bool more = un < NU, row = un % 9 == 0;
            if constexpr (NP == 3) {
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    if (more && i < 3) {
                        if (row) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                        else __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                    }
                }
            } else {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (more) {
                    if (row) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    else __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        read_barrier();
        const bool item_end = cc.tile + 1 >= cc.tend;
        if (item_end) {
            const int nb = cc.item % NCO, rest = cc.item / NCO;
            const int cb = rest % NCI, split = rest / NCI;
            const int ci = cb * 64 + wn * 32 + (lane & 31);
#pragma unroll
            for (int t = 0; t < 9; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int co = nb * 64 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    a.part[((size_t)(split * 9 + t) * a.Cout + co) * a.Cin + ci] = acc[t][r];
                    acc[t][r] = 0.f;
                }
        }
        advance(cc);
    }
}

// Persistent wgrad plan: about one item per CU (items = co blocks x ci blocks x splits)
void wgrad_x6w_plan(int ntiles, int Cout, int Cin, int cus, int& nsplit, int& tps) {
    const int64_t base = (int64_t)(Cout / 64) * (Cin / 64);
    int64_t ns = cdiv(cus, base);
    const int64_t per = (int64_t)9 * Cout * Cin * 4;  // fp32 partial slab per split
    int64_t cap = (192ll << 20) / per;
    if (cap < 1) cap = 1;
    if (ns > cap) ns = cap;
    if (ns > ntiles) ns = ntiles;
    if (ns < 1) ns = 1;
    tps = (int)cdiv(ntiles, ns);
    nsplit = (int)cdiv(ntiles, tps);
}

void launch_wgrad_x6(const WgradArgs& a, int np, hipStream_t st) {
    const int64_t items = (int64_t)(a.Cout / 64) * (a.Cin / 64) * a.nsplit;
    int64_t g = std::min<int64_t>(cu_count(st), (items + 7) / 8 * 8);
    g = std::max<int64_t>(8, g / 8 * 8);
    if (np == 3 && a.bn_y)  // (dy formed while loading; da may be absent with a route)
        hipLaunchKernelGGL((conv3x3_wgrad_x6w_kernel<WGX6W_TH, WGX6_TW, 3, 0, true>),
                           dim3((unsigned)g), dim3(512), 0, st, a);
    else if (np == 3)
        hipLaunchKernelGGL((conv3x3_wgrad_x6w_kernel<WGX6W_TH, WGX6_TW, 3>), dim3((unsigned)g),
                           dim3(512), 0, st, a);
    // bf16 storage of the activations (the host checked both sources alike) and of dy
    else if (a.src0 == nullptr && a.dy == nullptr)
        hipLaunchKernelGGL((conv3x3_wgrad_x6w_kernel<WGX6W_TH, WGX6_TW, 1, 3>),
                           dim3((unsigned)g), dim3(512), 0, st, a);
    else if (a.dy == nullptr)
        hipLaunchKernelGGL((conv3x3_wgrad_x6w_kernel<WGX6W_TH, WGX6_TW, 1, 2>),
                           dim3((unsigned)g), dim3(512), 0, st, a);
    else if (a.src0 == nullptr)
        hipLaunchKernelGGL((conv3x3_wgrad_x6w_kernel<WGX6W_TH, WGX6_TW, 1, 1>),
                           dim3((unsigned)g), dim3(512), 0, st, a);
    else
        hipLaunchKernelGGL((conv3x3_wgrad_x6w_kernel<WGX6W_TH, WGX6_TW, 1>), dim3((unsigned)g),
                           dim3(512), 0, st, a);
}

// Weight pack for the split path.  mode 0 (forward): GEMM N = Cout, K channels =
// Cin_pad; mode 1 (data gradient): N = Cin_pad, K channels = Cout, taps rotated
// by 180 degrees.  Layout [N/64][K/16][ky 3][piece 3][half 2][kx 3][64][8] bf16:
// the slab of one (column block, chunk, kernel row) is contiguous (18 KB) and
// equals one LDS weight stage of the kernels below.
__device__ __forceinline__ void pack_x6_elem(const float* w, __bf16* wpk, int Cin, int K,
                                             int mode, int np, int64_t e) {
    const int nchunk = K / 16;
    const int64_t plane = 3 * 64 * 8;  // one (ky, piece, half) sub-slab: kx x co x 8
    const int j = (int)(e & 7);
    int64_t r = e >> 3;
    const int co = (int)(r % 64);
    r /= 64;
    const int kx = (int)(r % 3);
    r /= 3;
    const int h = (int)(r % 2);
    r /= 2;
    const int ky = (int)(r % 3);
    r /= 3;
    const int chunk = (int)(r % nchunk), nb = (int)(r / nchunk);
    const int t = ky * 3 + kx;
    const int n = nb * 64 + co, k = chunk * 16 + h * 8 + j;
    float v;
    if (mode == 0) v = k < Cin ? w[((size_t)n * Cin + k) * 9 + t] : 0.f;
    else v = n < Cin ? w[((size_t)k * Cin + n) * 9 + (8 - t)] : 0.f;
    const __bf16 p0 = (__bf16)v;
    const float r1 = v - (float)p0;
    const __bf16 p1 = (__bf16)r1;
    const __bf16 p2 = (__bf16)(r1 - (float)p1);
    const size_t base = ((size_t)((nb * nchunk + chunk) * 3 + ky) * np * 2) * plane;
    const size_t off = ((size_t)kx * 64 + co) * 8 + j;
    wpk[base + (0 * 2 + h) * plane + off] = p0;
    if (np == 3) {
        wpk[base + (1 * 2 + h) * plane + off] = p1;
        wpk[base + (2 * 2 + h) * plane + off] = p2;
    }
}

__global__ void pack_x6_kernel(const float* w, __bf16* wpk, int Cout, int Cin, int N, int K,
                               int mode, int np) {
    (void)Cout;
    const int64_t total = (int64_t)N * K * 9;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x)
        pack_x6_elem(w, wpk, Cin, K, mode, np, e);
}

// The batched pack by (64-column block, 16-deep chunk) tiles: the tile's 64 x 16 x 9
// weights are read as contiguous OIHW runs into LDS (144 floats per output channel in
// the forward layout, 576 per input channel in the transposed data-gradient one), then
// written as whole 16-byte groups of 8 k-values per piece in the pack order.  Same
// element values and rounding as pack_x6_elem; the element-wise form read OIHW with a
// 36-byte lane stride (2.4x the algorithmic bytes per launch, profiles/r2h).
__global__ void __launch_bounds__(256) pack_x6_tile_kernel(PackBatch pb, int np) {
    int i = 0;
    while (i + 1 < pb.n && (int)blockIdx.x >= pb.first[i + 1]) ++i;  // uniform
    const PackItem& it = pb.item[i];
    const int mode = it.mode, Cin = it.Cin;
    const int K = mode == 0 ? it.Cin_pad : it.Cout, nchunk = K / 16;
    const int tb = (int)blockIdx.x - pb.first[i], nb = tb / nchunk, chunk = tb % nchunk;
    constexpr int RP = 145;  // row pitch (floats): odd, so the 64 rows hit distinct banks
    __shared__ float tile[64 * RP];  // [column n][k 0..15][tap t]
    const int tid = threadIdx.x;
    if (mode == 0) {
        // rows n = nb*64 + r: w[n][chunk*16 .. +16][0..8] = 144 contiguous floats
        for (int e = tid; e < 64 * 144; e += 256) {
            const int r = e / 144, c = e - r * 144;
            const bool ok = chunk * 16 + c / 9 < Cin;
            tile[r * RP + c] = ok ? it.w[((size_t)(nb * 64 + r) * Cin) * 9 + chunk * 144 + c] : 0.f;
        }
    } else {
        // rows k = chunk*16 + kk (output channels): w[k][nb*64 .. +64][0..8] = 576 floats,
        // stored at tap 8 - t (the rot180 of the data-gradient layout)
        for (int e = tid; e < 16 * 576; e += 256) {
            const int kk = e / 576, c = e - kk * 576, r = c / 9, ts = c - r * 9;
            const bool ok = nb * 64 + r < Cin;
            tile[r * RP + kk * 9 + (8 - ts)] =
                ok ? it.w[((size_t)(chunk * 16 + kk) * Cin) * 9 + nb * 576 + c] : 0.f;
        }
    }
    __syncthreads();
    constexpr int64_t plane = 3 * 64 * 8;
    __bf16* const out = static_cast<__bf16*>(it.wpk) + (size_t)((nb * nchunk + chunk) * 3) * np * 2 * plane;
    // units (ky, h, kx, co) of 8 k-values, co fastest: consecutive lanes, consecutive 16 B
    for (int u = tid; u < 3 * 2 * 3 * 64; u += 256) {
        const int co = u & 63, kx = (u >> 6) % 3, h = (u / 192) & 1, ky = u / 384;
        const float* src = tile + co * RP + h * 8 * 9 + ky * 3 + kx;
        unsigned short q0[8], q1[8], q2[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = src[j * 9];
            const __bf16 p0 = (__bf16)v;
            const float r1 = v - (float)p0;
            const __bf16 p1 = (__bf16)r1;
            const __bf16 p2 = (__bf16)(r1 - (float)p1);
            q0[j] = __builtin_bit_cast(unsigned short, p0);
            q1[j] = __builtin_bit_cast(unsigned short, p1);
            q2[j] = __builtin_bit_cast(unsigned short, p2);
        }
        auto pack8 = [](const unsigned short (&q)[8]) {
            u32x4 r;
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] = (unsigned)q[2 * k] | ((unsigned)q[2 * k + 1] << 16);
            return r;
        };
        const size_t off = (size_t)(kx * 64 + co) * 8;
        __bf16* o = out + (size_t)ky * np * 2 * plane + (size_t)h * plane + off;
        *reinterpret_cast<u32x4*>(o) = pack8(q0);
        if (np == 3) {
            *reinterpret_cast<u32x4*>(o + 2 * plane) = pack8(q1);
            *reinterpret_cast<u32x4*>(o + 4 * plane) = pack8(q2);
        }
    }
}

// Forward / data-gradient form by shape (no runtime knobs: the form, its tiling and hence
// the BatchNorm slot count are functions of the shape and the piece count):
//  - images >= 32 wide: conv3x3_fwd_x6r_kernel, 8 x 32-pixel items (16x16x32 MFMA tiles
//    for split-bf16, 32x32x16 for single-piece bf16);
//  - split-bf16 images 16-31 wide: the same with 8 x 16-pixel items, so that bs16's
//    16-wide layers have 256 items for 256 CUs (152-166 -> 216-223 TF/s vs the
//    single-stage kernel);
//  - narrower images (and single-piece ones < 32 wide): conv3x3_fwd_x6_kernel, 8 x 16-pixel
//    tiles, one workgroup per tile.
// Measured and dropped (round 2): 16 x 16 items for the 16-wide layers, the 32x32x16 form
// for split-bf16, 512-pixel single-piece items, two compute waves per SIMD.
// (the single-piece persistent form also takes 16-wide images of even height: x6_fwd_form)
static bool use_x6r(int W, int np) { return W >= 32 || (np == 3 && W >= 16); }
static bool np1_w16(int H, int W) { return W == 16 && H % 2 == 0; }
//  - single-piece (bf16) images >= 32 wide: 256 x 128 items (8 x 32 pixels, two 64-column
//    weight slabs) where N is a multiple of 128, 512 x 64 items (16 x 32 pixels) where
//    N = 64 -- each compute wave 4 x 2 MFMA tiles, 0.75 LDS fragment reads per MFMA
//    instead of 1.25 -- unless that leaves fewer items than a 256-CU device has: then the
//    256 x 64 items.  The plan assumes 256 CUs whatever the device, so the BatchNorm
//    partial order (the slot layout) is a function of the shape only.
X6Form x6_fwd_form(int B, int H, int W, int K, int N, int np) {
    if (np == 3) {
        if (W >= 32) return {8, 32, 1, 2, true};
        if (W >= 16) return {8, 16, 1, 2, true};
        return {8, 16, 1, 1, false};
    }
#ifndef X6R_NP1_W16  // (A/B builds: -D X6R_NP1_W16=0 keeps the single-stage kernel)
#define X6R_NP1_W16 1
#endif
    // 16-wide images: 8 x 16 items (128 pixels; two image rows per 32-pixel MFMA tile), so
    // bs16 x 16^2 x 512 channels is 256 items -- one per CU (round 6)
    if (X6R_NP1_W16 && np1_w16(H, W)) return {8, 16, 1, 2, true};
    if (W < 32) return {8, 16, 1, 1, false};
#ifdef X6R_NO_WIDE  // A/B build: the 256 x 64 items everywhere
    return {8, 32, 1, 2, true};
#endif
    constexpr int64_t kPlanCUs = 256;
    const int64_t tiles8 = (int64_t)B * cdiv(H, 8) * cdiv(W, 32);
    const int64_t tiles16 = (int64_t)B * cdiv(H, 16) * cdiv(W, 32);
    if (N % 128 == 0 && tiles8 * (N / 128) >= kPlanCUs) return {8, 32, 2, 2, true};
    // 512 x 64 items only where an item runs >= 16 K steps: with fewer the doubled
    // per-item epilogue costs more than the halved fragment reads save (in-process A/B
    // against 256 x 64 everywhere, profiles/r5b_ab_wide_forms_bf16.txt: K = 256 -3 %,
    // K = 64/128 +4-10 %)
    if (N % 128 != 0 && K >= 256 && tiles16 * (N / 64) >= kPlanCUs) return {16, 32, 1, 4, true};
    return {8, 32, 1, 2, true};
}
int fwd_x6_stat_slots(const X6Form& f, int B, int H, int W) {
    const int ntiles = (int)(B * cdiv(H, f.th) * cdiv(W, f.tw));
    return f.persistent ? f.wm * ntiles : ntiles;  // persistent forms: one slot per pixel group
}

// ---------------------------------------------------------------------------
// Image layer (inc.conv_op.0: a 3-channel image zero-extended to 8 channels, one
// 16-channel K chunk, 64 outputs) as a direct fp32-FMA convolution.  Through x6r each
// 256-pixel item is a single K chunk, so its pipeline prologue and epilogue dominate
// (113-128 us at bs16 x 256^2 against 38 us of output stores).  The layer is bound by
// store issue, so the mapping is chosen for the stores: 16 lanes hold one pixel's 64
// channels (4 each), a wave's four 16-lane groups are four 16-pixel row segments, and
// every store instruction writes four whole 256-B pixels.  A persistent workgroup
// rebuilds the fp32 weights once from the split-bf16 pack (p0 + p1 + p2 == w exactly)
// and finds the highest input channel with a nonzero weight (the zero padding is
// skipped), then walks 8 x 32-pixel tiles, fetching the next tile's halo into
// registers while the current one computes; the halo sits channel-planar in LDS so a
// segment's 18 inputs are 4 ds_read_b128 + 1 ds_read_b64, reused over the 3 kx taps.
// Products and sums in fp32 (the fp32-MFMA path's arithmetic class), as packed pairs.
// Epilogue: bias, store, BatchNorm partials (count, sum, M2 about the slot mean) in
// x6r's slot layout (NWM row groups per tile).
template <int NWM, int PX, bool WF32>
__global__ void __launch_bounds__(4096 / PX) conv3x3_img_fwd_kernel(ConvFwdArgs a) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    // PX pixels per thread: 16 lanes x (TW / PX) segments per tile row
    constexpr int NT = 4096 / PX, NWV = NT / 64, RPW = 4 * PX / 32;  // rows per wave
    constexpr int TH = 8, TW = 32, HWP = 36, HROWS = TH + 2, CIN = 8;
    constexpr int NH = HROWS * (TW + 2) * 2;     // halo f32x4 pieces (2 per pixel)
    constexpr int HPT = (NH + NT - 1) / NT;      // per thread
    __shared__ float wsm[9 * CIN][64];           // [tap * 8 + ci][co]
    __shared__ float xs[2][CIN][HROWS * HWP];    // channel-planar halo, double-buffered
    __shared__ float wred[2][NWV][64];           // per-wave channel sums / M2 partials
    __shared__ int nci_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tpi = a.tiles_x * a.tiles_y;
    // output channels 64*nb .. 64*nb+63 of Cout = 64 * gridDim.y (64 or 128)
    const int nb = blockIdx.y, n0 = 64 * nb;
    // lazy BN+ReLU of the source (the image itself has none): this thread's 4 channels
    // are fixed (piece q = tid & 1, NT even); zero padding stays zero
    const bool aon = a.sc0 != nullptr;
    f32x4 asc = {1.f, 1.f, 1.f, 1.f}, ash = {0.f, 0.f, 0.f, 0.f};
    if (aon)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            asc[i] = a.sc0[4 * (tid & 1) + i];
            ash[i] = a.sh0[4 * (tid & 1) + i];
        }
    auto halo_fetch = [&](int tile, f32x4* r, unsigned& hv) {
        const int b = tile / tpi, trem = tile % tpi;
        const int ty0 = (trem / a.tiles_x) * TH, tx0 = (trem % a.tiles_x) * TW;
        hv = 0u;
#pragma unroll
        for (int k = 0; k < HPT; ++k) {
            const int e = tid + NT * k, hp = e >> 1, q = e & 1;
            const int gy = ty0 - 1 + hp / (TW + 2), gx = tx0 - 1 + hp % (TW + 2);
            r[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (e < NH && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
                r[k] = *reinterpret_cast<const f32x4*>(
                    a.src0 + ((size_t)(b * a.H + gy) * a.W + gx) * CIN + 4 * q);
                hv |= 1u << k;
            }
        }
    };
    auto halo_put = [&](int buf, const f32x4* r, unsigned hv) {
#pragma unroll
        for (int k = 0; k < HPT; ++k) {
            const int e = tid + NT * k, hp = e >> 1, q = e & 1;
            const int o = (hp / (TW + 2)) * HWP + hp % (TW + 2);
            const bool act = aon && ((hv >> k) & 1u);
            if (e < NH)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    xs[buf][4 * q + i][o] = act ? fmaxf(fmaf(r[k][i], asc[i], ash[i]), 0.f) : r[k][i];
        }
    };
    if (blockIdx.x >= a.ntiles) return;
    f32x4 hr[HPT];
    unsigned hv;
    halo_fetch(blockIdx.x, hr, hv);
    // weights: pack layout of pack_x6_elem (mode 0, K = 16, nb = 0)
    const __bf16* wp = static_cast<const __bf16*>(a.wpk) + (size_t)nb * 3 * 6 * (3 * 64 * 8);
    constexpr int plane = 3 * 64 * 8;
    if (tid == 0) nci_s = 0;
    __syncthreads();
    int hi = 0;
    if constexpr (WF32) {
        // fp32 pack [K/8][9][N][8] (K = 8): element (t, co, ci) at (t*64 + co)*8 + ci
        constexpr int NE = 9 * CIN * 64 / NT;
        const float* wf = static_cast<const float*>(a.wpk);
        float pv[NE];
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const int e = tid + NT * k, ci = e & 7, co = (e >> 3) & 63, t = e >> 9;
            pv[k] = wf[((size_t)t * a.Cout + n0 + co) * 8 + ci];
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const int e = tid + NT * k, ci = e & 7, co = (e >> 3) & 63, t = e >> 9;
            wsm[t * CIN + ci][co] = pv[k];
            if (pv[k] != 0.f) hi = max(hi, ci + 1);
        }
    } else {
        // all 3 x 9 * 512 / NT loads issued before the first is used (one round trip)
        constexpr int NE = 9 * CIN * 64 / NT;
        __bf16 pc[NE][3];
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const int e = tid + NT * k, ci = e & 7, co = (e >> 3) & 63, t = e >> 9;
            const size_t base = (size_t)(t / 3) * 6 * plane + ((size_t)(t % 3) * 64 + co) * 8 + ci;
#pragma unroll
            for (int q = 0; q < 3; ++q) pc[k][q] = wp[base + 2 * q * plane];
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const int e = tid + NT * k, ci = e & 7, co = (e >> 3) & 63, t = e >> 9;
            const float v = ((float)pc[k][0] + (float)pc[k][1]) + (float)pc[k][2];
            wsm[t * CIN + ci][co] = v;
            if (v != 0.f) hi = max(hi, ci + 1);
        }
    }
    for (int o = 32; o > 0; o >>= 1) hi = max(hi, __shfl_xor(hi, o, 64));
    if (lane == 0) atomicMax(&nci_s, hi);
    halo_put(0, hr, hv);
    __syncthreads();
    const int nci = nci_s;
    // thread: channels 4*cq..+3 of the PX-pixel row segment (row, c0..c0+PX-1)
    constexpr int SPR = TW / PX;  // segments per row
    const int cq = lane & 15, seg = tid >> 4, row = seg / SPR, c0 = (seg % SPR) * PX;
    constexpr int RPS = TH / NWM;  // rows per BN slot
    constexpr int WPS = RPS / RPW; // waves per BN slot
    int buf = 0;
    for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x, buf ^= 1) {
        const int nxt = tile + gridDim.x;
        if (nxt < a.ntiles) halo_fetch(nxt, hr, hv);
        const int b = tile / tpi, trem = tile % tpi;
        const int ty0 = (trem / a.tiles_x) * TH, tx0 = (trem % a.tiles_x) * TW;
        f2 acc[PX][2];
#pragma unroll
        for (int p = 0; p < PX; ++p) acc[p][0] = acc[p][1] = f2{0.f, 0.f};
        for (int ky = 0; ky < 3; ++ky) {
            for (int ci = 0; ci < nci; ++ci) {
                const float* xr = &xs[buf][ci][(row + ky) * HWP + c0];
                float x[PX + 2];
#pragma unroll
                for (int k = 0; k < PX / 4; ++k) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + 4 * k);
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[4 * k + i] = v[i];
                }
                {
                    const f2 v = *reinterpret_cast<const f2*>(xr + PX);
                    x[PX] = v.x;
                    x[PX + 1] = v.y;
                }
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const f32x4 wv = *reinterpret_cast<const f32x4*>(&wsm[(3 * ky + kx) * CIN + ci][4 * cq]);
                    const f2 w01 = f2{wv[0], wv[1]}, w23 = f2{wv[2], wv[3]};
#pragma unroll
                    for (int p = 0; p < PX; ++p) {
                        const f2 xv = f2{x[p + kx], x[p + kx]};
                        acc[p][0] = __builtin_elementwise_fma(xv, w01, acc[p][0]);
                        acc[p][1] = __builtin_elementwise_fma(xv, w23, acc[p][1]);
                    }
                }
            }
        }
        // bias, store (16 lanes = one whole pixel), per-thread sums over valid pixels
        const int vh = min(TH, a.H - ty0), vw = min(TW, a.W - tx0);
        const bool rok = row < vh;
        f32x4 bv = {0.f, 0.f, 0.f, 0.f};
        if (a.bias)
#pragma unroll
            for (int i = 0; i < 4; ++i) bv[i] = a.bias[n0 + 4 * cq + i];
        const size_t orow = ((size_t)(b * a.H + ty0 + row) * a.W + tx0 + c0) * a.Cout + n0 + 4 * cq;
        // out0 == nullptr: bf16 storage only, the statistics describe the rounded values
        const bool only16 = a.out0 == nullptr;
        float sj[4] = {0.f, 0.f, 0.f, 0.f};
        float v[PX][4];
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            v[p][0] = acc[p][0].x + bv[0];
            v[p][1] = acc[p][0].y + bv[1];
            v[p][2] = acc[p][1].x + bv[2];
            v[p][3] = acc[p][1].y + bv[3];
            if (only16)
#pragma unroll
                for (int i = 0; i < 4; ++i) v[p][i] = (float)(__bf16)v[p][i];
            if (rok && c0 + p < vw) {
#ifndef IMG_NOSTORE
                if (!only16)
                    *reinterpret_cast<f32x4*>(a.out0 + orow + (size_t)p * a.Cout) =
                        f32x4{v[p][0], v[p][1], v[p][2], v[p][3]};
                if (a.out0_16) {
                    typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
                    *reinterpret_cast<bf4*>(a.out0_16 + orow + (size_t)p * a.Cout) =
                        bf4{(__bf16)v[p][0], (__bf16)v[p][1], (__bf16)v[p][2], (__bf16)v[p][3]};
                }
#endif
#pragma unroll
                for (int i = 0; i < 4; ++i) sj[i] += v[p][i];
            }
        }
        if (nxt < a.ntiles) halo_put(buf ^ 1, hr, hv);
        if (a.stats != nullptr) {
            // BatchNorm partials per (channel, slot): slot = NWM * tile + row group.
            // wave sums: the 4 segments holding the same channels (lane bits 4, 5)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                sj[i] += __shfl_xor(sj[i], 16, 64);
                sj[i] += __shfl_xor(sj[i], 32, 64);
            }
            if (lane < 16)
#pragma unroll
                for (int i = 0; i < 4; ++i) wred[0][wave][4 * cq + i] = sj[i];
            __syncthreads();
            const int sl = row / RPS, w0 = sl * WPS;
            const int rows = min(max(vh - sl * RPS, 0), RPS);
            const float cnt = (float)(rows * vw);
            float qj[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float s = 0.f;
#pragma unroll
                for (int k = 0; k < WPS; ++k) s += wred[0][w0 + k][4 * cq + i];
                const float mu = cnt > 0.f ? s / cnt : 0.f;
                float q = 0.f;
#pragma unroll
                for (int p = 0; p < PX; ++p) {
                    const float d = v[p][i] - mu;
                    if (rok && c0 + p < vw) q = fmaf(d, d, q);
                }
                q += __shfl_xor(q, 16, 64);
                q += __shfl_xor(q, 32, 64);
                qj[i] = q;
            }
            if (lane < 16)
#pragma unroll
                for (int i = 0; i < 4; ++i) wred[1][wave][4 * cq + i] = qj[i];
            __syncthreads();
            if (tid < 64 * NWM) {
                const int c = tid & 63, s2 = tid >> 6;
                float sum = 0.f, m2 = 0.f;
                for (int k = 0; k < WPS; ++k) {
                    sum += wred[0][s2 * WPS + k][c];
                    m2 += wred[1][s2 * WPS + k][c];
                }
                const int rows2 = min(max(vh - s2 * RPS, 0), RPS);
                const size_t S = (size_t)NWM * a.ntiles, slot = (size_t)NWM * tile + s2;
                a.stats[(0 * (size_t)a.Cout + n0 + c) * S + slot] = (float)(rows2 * vw);
                a.stats[(1 * (size_t)a.Cout + n0 + c) * S + slot] = sum;
                a.stats[(2 * (size_t)a.Cout + n0 + c) * S + slot] = m2;
            }
        }
        __syncthreads();  // halo buffer swap; wred reuse
    }
}

#ifndef IMG_PX
#define IMG_PX 8
#endif
#ifndef IMG_BPC
#define IMG_BPC 2
#endif

bool img_fwd_eligible(int W, int C0, int C1, int Cout) {
    // PGUNet4's image layer is 3 -> 64, PGUNet3's 3 -> 128 (two 64-channel column blocks)
    return W >= 32 && C0 == 8 && C1 == 0 && (Cout == 64 || Cout == 128);
}
int img_fwd_slots(int B, int H, int W, int nwm) {
    return nwm * B * (int)cdiv(H, 8) * (int)cdiv(W, 32);
}

// the image layer's direct fp32 kernel (8 x 32 tiles; a.tiles_* / ntiles set for them);
// false when the call does not qualify
bool launch_img_fwd(const ConvFwdArgs& a, bool wf32, hipStream_t st) {
    if (!img_fwd_eligible(a.W, a.C0, a.C1, a.Cout) || a.split != a.Cout || a.acc0 ||
        a.bnb_part)
        return false;
    // persistent: IMG_BPC workgroups per CU
    int64_t g = std::min<int64_t>(IMG_BPC * (int64_t)cu_count(st), (int64_t)a.ntiles);
    g = std::max<int64_t>(1, g);
    constexpr int PX = IMG_PX;
    const dim3 grid((unsigned)g, (unsigned)(a.Cout / 64)), block(4096 / PX);
    if (wf32)
        hipLaunchKernelGGL((conv3x3_img_fwd_kernel<2, PX, true>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((conv3x3_img_fwd_kernel<2, PX, false>), grid, block, 0, st, a);
    return true;
}

#ifndef X6R_RES_ON  // (A/B builds: -D X6R_RES_ON=0 streams the weight rows as before)
#define X6R_RES_ON 1
#endif
int launch_fwd_x6(const ConvFwdArgs& a, int np, hipStream_t st) {
    const X6Form f = x6_fwd_form(a.B, a.H, a.W, a.Cin, a.Cout, np);
    const int64_t items = (int64_t)a.ntiles * (a.Cout / (64 * f.nslab));
    if (np == 3 && use_x6r(a.W, np) && a.Cin == 16 && launch_img_fwd(a, false, st))
        return FWD_WROTE_OUT16;
    if (use_x6r(a.W, np) || (np == 1 && f.persistent)) {
        // persistent: one workgroup per CU (a multiple of 8: blockIdx % 8 = XCD), each
        // walking a strided share of its XCD's contiguous item range
        int64_t g = std::min<int64_t>(cu_count(st), (items + 7) / 8 * 8);
        g = std::max<int64_t>(8, g / 8 * 8);
        if (np == 3 && a.W < 32)
            hipLaunchKernelGGL((conv3x3_fwd_x6r_kernel<3, true, 16, 8>), dim3((unsigned)g),
                               dim3(512), 0, st, a);
        else if (np == 3)
            hipLaunchKernelGGL((conv3x3_fwd_x6r_kernel<3, true>), dim3((unsigned)g), dim3(512), 0,
                               st, a);
        else {
            const bool xb16 = !a.src0 && a.src0_16 && (a.C1 == 0 || (!a.src1 && a.src1_16));
            const dim3 grid((unsigned)g), block(512);
            // the 4 x 2-tile forms fuse the BatchNorm-backward partials of a bf16 y only
            // (x6_epilogue_wave Y32); with an fp32 y the caller's reduction pass writes them
            ConvFwdArgs b = a;
            const bool wide = f.nslab == 2 || f.th == 16;
            const bool nofuse = wide && a.bnb_part && !a.bnb_y.h;
            if (nofuse) b.bnb_part = nullptr;
            if (f.tw == 16) {  // (16-wide sources are fp32: ugpg_conv3x3_fwd)
                hipLaunchKernelGGL((conv3x3_fwd_x6r_kernel<1, false, 16, 8, false>), grid, block, 0, st, b);
            } else if (f.nslab == 2 || f.th == 16) {
                // the 4 x 2-tile forms: whole-line bf16 stores when the output allows them
                // (with BN-backward partials: of a bf16 y, DMA'd into the staging areas)
                const bool pair = X6R_PAIR16 && b.out0 == nullptr && b.out0_16 != nullptr &&
                                  (b.bnb_part == nullptr || (X6R_PAIR16_BNB && b.bnb_y.h)) && !b.acc0 &&
                                  b.split == b.Cout && b.W % 32 == 0;
                const int pr = !pair ? 0 : b.bnb_part ? 2 : 1;
#define X6R_LW(TH_, XB_, NS_, PR_) \
    hipLaunchKernelGGL((conv3x3_fwd_x6r_kernel<1, false, 32, TH_, XB_, NS_, false, PR_>), grid, block, 0, st, b)
#define X6R_LW3(TH_, XB_, NS_) \
    do { if (pr == 2) X6R_LW(TH_, XB_, NS_, 2); else if (pr == 1) X6R_LW(TH_, XB_, NS_, 1); \
         else X6R_LW(TH_, XB_, NS_, 0); } while (0)
                if (f.nslab == 2) {
                    if (xb16) X6R_LW3(8, true, 2);
                    else X6R_LW3(8, false, 2);
                } else {
                    if (xb16) X6R_LW3(16, true, 1);
                    else X6R_LW3(16, false, 1);
                }
#undef X6R_LW3
#undef X6R_LW
            } else if (X6R_RES_ON && a.Cin == 64 && a.Cout == 64) {  // resident weights
                if (xb16) hipLaunchKernelGGL((conv3x3_fwd_x6r_kernel<1, false, 32, 8, true, 1, true>), grid, block, 0, st, b);
                else hipLaunchKernelGGL((conv3x3_fwd_x6r_kernel<1, false, 32, 8, false, 1, true>), grid, block, 0, st, b);
            } else {
                if (xb16) hipLaunchKernelGGL((conv3x3_fwd_x6r_kernel<1, false, 32, 8, true>), grid, block, 0, st, b);
                else hipLaunchKernelGGL((conv3x3_fwd_x6r_kernel<1, false, 32, 8, false>), grid, block, 0, st, b);
            }
            return (nofuse ? 0 : FWD_WROTE_BNB) | FWD_WROTE_OUT16;
        }
        // every persistent form fuses the BatchNorm-backward partials into its epilogue
        return FWD_WROTE_BNB;
    }
    // single-stage kernel: 8 x 16-pixel tiles (fwd_x6_tile_*)
    const unsigned grid = (unsigned)items;
    if (np == 3)
        hipLaunchKernelGGL((conv3x3_fwd_x6_kernel<8, 16, true, 3>), dim3(grid), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((conv3x3_fwd_x6_kernel<8, 16, true, 1>), dim3(grid), dim3(256), 0, st, a);
    return 0;
}

void launch_pack_x6(const float* w, void* wpk, int Cout, int Cin, int Cin_pad, int mode, int np,
                    hipStream_t st) {
    const int N = mode == 0 ? Cout : Cin_pad, K = mode == 0 ? Cin_pad : Cout;
    hipLaunchKernelGGL(pack_x6_kernel, dim3(stream_grid((int64_t)N * K * 9)), dim3(256), 0, st, w,
                       static_cast<__bf16*>(wpk), Cout, Cin, N, K, mode, np);
}

void launch_pack_x6_batch(const PackItem* items, int n, int np, hipStream_t st) {
    for (int i0 = 0; i0 < n; i0 += PACK_BATCH_MAX) {
        PackBatch pb;
        pb.n = std::min(PACK_BATCH_MAX, n - i0);
        int blocks = 0;
        for (int i = 0; i < pb.n; ++i) {
            const PackItem& it = items[i0 + i];
            pb.item[i] = it;
            pb.first[i] = blocks;
            const int N = it.mode == 0 ? it.Cout : it.Cin_pad, K = it.mode == 0 ? it.Cin_pad : it.Cout;
            blocks += (N / 64) * (K / 16);  // one workgroup per (64-column, 16-deep) tile
        }
        pb.first[pb.n] = blocks;
        hipLaunchKernelGGL(pack_x6_tile_kernel, dim3((unsigned)blocks), dim3(256), 0, st, pb, np);
    }
}

}  // namespace ugpg
