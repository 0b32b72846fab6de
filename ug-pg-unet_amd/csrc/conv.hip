#include <vector>
// 3x3 / pad-1 convolution for gfx950: forward, data-gradient (same kernel with a
// rotated/transposed weight pack) and weight-gradient, all NHWC fp32 on
// v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains, 157 TF/s peak).
//
// Replaces aten::convolution / convolution_backward behind DoubleConv
// (reference UG_unet_parts.py:10,13).
//
// Forward tile: a TH x TW output-pixel rectangle x BN output channels.  Per input
// channel chunk (BKC channels) the (TH+2)x(TW+2) halo and the 9 x BKC x BN weight
// slab are staged in LDS once and reused by all 9 taps (9x reuse of every loaded
// activation).  The consumer-side BatchNorm+ReLU of the producing layer is applied
// while staging (lazy activation), so the normalised tensor never touches HBM, and
// zero padding stays zero.  The epilogue adds the bias, stores, and emits per-tile
// (count, sum, M2) BatchNorm partials (two-pass inside the tile, Chan-merged later).
//
// MFMA k-permutation: lane l (h = l>>5) feeds k-slot h of step s with input channel
// 8g + 4h + s for both operands, so each lane's 4 consecutive channels come from one
// 16-byte ds_read_b128 for A and one for B.
#include "conv_common.h"

namespace ugpg {


template <int TH, int TW, int BN, int BKC, int WM, int WN, int MINW = 1>
__global__ void __launch_bounds__(256, MINW) conv3x3_fwd_kernel(ConvFwdArgs a) {
    constexpr int BM = TH * TW, HWD = TW + 2, NHALO = (TH + 2) * HWD;
    constexpr int WTM = BM / WM, WTN = BN / WN, MT = WTM / 32, NT = WTN / 32;
    constexpr int AP = BKC + 4;  // +16 B per halo pixel: spreads ds_read_b128 over banks
    constexpr int G = BKC / 8;
    constexpr int A_VEC = NHALO * BKC / 4, B_VEC = 9 * G * BN * 2;
    constexpr int A_PER = (A_VEC + 255) / 256, B_PER = (B_VEC + 255) / 256;
    static_assert(WM * WN == 4 && MT >= 1 && NT >= 1 && A_PER <= 32, "bad tile");
    __shared__ __attribute__((aligned(16))) float smem[NHALO * AP + 9 * G * BN * 8];
    float* As = smem;
    float* Bs = smem + NHALO * AP;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int NB = a.Cout / BN;
    const int nb = blockIdx.x % NB, tile = blockIdx.x / NB;
    const int n0 = nb * BN;
    const int tpi = a.tiles_x * a.tiles_y;
    const int b = tile / tpi, trem = tile % tpi;
    const int ty0 = (trem / a.tiles_x) * TH, tx0 = (trem % a.tiles_x) * TW;

    f32x4 ra[A_PER];
    f32x4 rb[B_PER];
    unsigned avalid = 0;
    Act4 ract;  // coefficients of this thread's 4 channels (fixed: q = tid % (BKC/4))
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
        aon = sc != nullptr;
        ract = act_load4(sc, sh, cb + (tid % (BKC / 4)) * 4);
        avalid = 0;
#pragma unroll
        for (int v = 0; v < A_PER; ++v) {
            const int idx = tid + v * 256;
            f32x4 val = {0.f, 0.f, 0.f, 0.f};
            if (idx < A_VEC) {
                const int hp = idx / (BKC / 4), q = idx % (BKC / 4);
                const int gy = ty0 - 1 + hp / HWD, gx = tx0 - 1 + hp % HWD;
                if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
                    val = *reinterpret_cast<const f32x4*>(
                        src + ((size_t)(b * a.H + gy) * a.W + gx) * Cs + cb + q * 4);
                    avalid |= 1u << v;
                }
            }
            ra[v] = val;
        }
        const float* wsrc = static_cast<const float*>(a.wpk) + (size_t)c * G * 9 * a.Cout * 8;
#pragma unroll
        for (int v = 0; v < B_PER; ++v) {
            const int idx = tid + v * 256;
            if (idx < B_VEC) {
                const int t = idx / (G * BN * 2), g = (idx / (BN * 2)) % G, r2 = idx % (BN * 2);
                rb[v] = *reinterpret_cast<const f32x4*>(
                    wsrc + ((size_t)(g * 9 + t) * a.Cout + n0) * 8 + r2 * 4);
            }
        }
    };

    auto lstore = [&](int c) {
        (void)c;
#pragma unroll
        for (int v = 0; v < A_PER; ++v) {
            const int idx = tid + v * 256;
            if (idx < A_VEC) {
                const int hp = idx / (BKC / 4), q = idx % (BKC / 4);
                f32x4 val = ra[v];
                if ((avalid >> v) & 1u) val = act_reg4(val, ract, aon);
                *reinterpret_cast<f32x4*>(&As[hp * AP + q * 4]) = val;
            }
        }
#pragma unroll
        for (int v = 0; v < B_PER; ++v) {
            const int idx = tid + v * 256;
            if (idx < B_VEC) *reinterpret_cast<f32x4*>(&Bs[idx * 4]) = rb[v];
        }
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    int aoff[MT], boff[NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = wm * WTM + mt * 32 + (lane & 31);
        aoff[mt] = ((m / TW) * HWD + (m % TW)) * AP + 4 * (lane >> 5);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) boff[nt] = (wn * WTN + nt * 32 + (lane & 31)) * 8 + 4 * (lane >> 5);

    // fragment loads of step i (= tap t, channel group g): A from the halo, B from the slab
    constexpr int NSTEP = 9 * G;
    auto ldfrag = [&](int i, f32x4* af, f32x4* bf) {
        const int t = i / G, g = i % G;
        const int toff = ((t / 3) * HWD + (t % 3)) * AP + g * 8;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
            af[mt] = *reinterpret_cast<const f32x4*>(&As[aoff[mt] + toff]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
            bf[nt] = *reinterpret_cast<const f32x4*>(&Bs[i * BN * 8 + boff[nt]]);
    };

    const int nchunk = a.Cin / BKC;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int c = 0; c < nchunk; ++c) {
        if (c + 1 < nchunk) gload(c + 1);
        // software-pipelined: step i+1's ds_reads are in flight under step i's MFMAs
        f32x4 fa[2][MT], fb[2][NT];
        ldfrag(0, fa[0], fb[0]);
#pragma unroll
        for (int i = 0; i < NSTEP; ++i) {
            if (i + 1 < NSTEP) ldfrag(i + 1, fa[(i + 1) & 1], fb[(i + 1) & 1]);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                            fa[i & 1][mt][s], fb[i & 1][nt][s], acc[mt][nt], 0, 0, 0);
        }
        __syncthreads();
        if (c + 1 < nchunk) {
            lstore(c + 1);
            __syncthreads();
        }
    }

    conv_epilogue<TH, TW, BN, WM, WN, MT, NT, false>(a, acc, smem, tile, b, ty0, tx0, n0, wm, wn);
}

// ---------------------------------------------------------------------------
// Weight gradient: per block a 64 (co) x 64 (ci) x 9 (tap) output, 4 waves as
// 2 (co) x 2 (ci) each owning nine 32x32 accumulators; reduction over the pixel
// tiles of one split.  Operands from LDS: dy tile [P][64], activated input halo
// [(TH+2)(TW+2)][64]; one MFMA k-step = 2 pixels.
// ---------------------------------------------------------------------------

template <int TH, int TW>
__global__ void __launch_bounds__(256) conv3x3_wgrad_kernel(WgradArgs a) {
    constexpr int P = TH * TW, HWD = TW + 2, NHALO = (TH + 2) * HWD;
    constexpr int DY_VEC = P * 16, X_VEC = NHALO * 16;
    constexpr int DY_PER = (DY_VEC + 255) / 256, X_PER = (X_VEC + 255) / 256;
    static_assert(X_PER <= 32, "halo too large");
    __shared__ __attribute__((aligned(16))) float smem[(P + NHALO) * 64];
    float* dys = smem;
    float* xs = smem + P * 64;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int NCO = a.Cout / 64, NCI = (a.Cin + 63) / 64;
    const int nb = blockIdx.x % NCO;
    const int rest = blockIdx.x / NCO;
    const int cb = rest % NCI, split = rest / NCI;
    const int co0 = nb * 64, ci0 = cb * 64;
    const int t_begin = split * a.tps, t_end = min(a.ntiles, t_begin + a.tps);

    const float* xsrc = a.src0;
    const float* xsc = a.sc0;
    const float* xsh = a.sh0;
    int Cs = a.C0, cbase = ci0;
    if (ci0 >= a.C0) {
        xsrc = a.src1;
        xsc = a.sc1;
        xsh = a.sh1;
        Cs = a.C1;
        cbase = ci0 - a.C0;
    }
    const int tpi = a.tiles_x * a.tiles_y;
    const Act4 xact = act_load4(xsc, xsh, cbase + (tid & 15) * 4);  // q = idx & 15 = tid & 15
    const bool xon = xsc != nullptr;

    f32x4 rdy[DY_PER], rx[X_PER];
    unsigned xvalid = 0;
    auto gload = [&](int tile) {
        const int b = tile / tpi, trem = tile % tpi;
        const int ty0 = (trem / a.tiles_x) * TH, tx0 = (trem % a.tiles_x) * TW;
#pragma unroll
        for (int v = 0; v < DY_PER; ++v) {
            const int idx = tid + v * 256;
            f32x4 val = {0.f, 0.f, 0.f, 0.f};
            if (idx < DY_VEC) {
                const int p = idx >> 4, q = idx & 15;
                const int gy = ty0 + p / TW, gx = tx0 + p % TW;
                if (gy < a.H && gx < a.W)
                    val = *reinterpret_cast<const f32x4*>(
                        a.dy + ((size_t)(b * a.H + gy) * a.W + gx) * a.Cout + co0 + q * 4);
            }
            rdy[v] = val;
        }
        xvalid = 0;
#pragma unroll
        for (int v = 0; v < X_PER; ++v) {
            const int idx = tid + v * 256;
            f32x4 val = {0.f, 0.f, 0.f, 0.f};
            if (idx < X_VEC) {
                const int hp = idx >> 4, q = idx & 15;
                const int gy = ty0 - 1 + hp / HWD, gx = tx0 - 1 + hp % HWD;
                if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W && cbase + q * 4 < Cs) {
                    val = *reinterpret_cast<const f32x4*>(
                        xsrc + ((size_t)(b * a.H + gy) * a.W + gx) * Cs + cbase + q * 4);
                    xvalid |= 1u << v;
                }
            }
            rx[v] = val;
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int v = 0; v < DY_PER; ++v) {
            const int idx = tid + v * 256;
            if (idx < DY_VEC) *reinterpret_cast<f32x4*>(&dys[idx * 4]) = rdy[v];
        }
#pragma unroll
        for (int v = 0; v < X_PER; ++v) {
            const int idx = tid + v * 256;
            if (idx < X_VEC) {
                f32x4 val = rx[v];
                if ((xvalid >> v) & 1u) val = act_reg4(val, xact, xon);
                *reinterpret_cast<f32x4*>(&xs[idx * 4]) = val;
            }
        }
    };

    f32x16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    float dbacc = 0.f;
    const bool do_db = (a.dbpart != nullptr) && cb == 0 && tid < 64;

    if (t_begin < t_end) gload(t_begin);
    for (int tile = t_begin; tile < t_end; ++tile) {
        __syncthreads();
        lstore();
        __syncthreads();
        if (tile + 1 < t_end) gload(tile + 1);
        const int arow = wm * 32 + (lane & 31), bcol = wn * 32 + (lane & 31);
        // k-step ks = pixels 2ks, 2ks+1; fragments of step ks+1 prefetched under step ks
        auto ldk = [&](int ks, float& af, float* bf) {
            const int p = 2 * ks + (lane >> 5);
            af = dys[p * 64 + arow];
            const int hb = ((p / TW) * HWD + (p % TW)) * 64 + bcol;
#pragma unroll
            for (int t = 0; t < 9; ++t) bf[t] = xs[hb + ((t / 3) * HWD + (t % 3)) * 64];
        };
        static_assert((P / 2) % 2 == 0, "two-step body needs an even k-step count");
        float a0, a1, b0[9], b1[9];
        ldk(0, a0, b0);
#pragma unroll 1
        for (int ks = 0; ks < P / 2; ks += 2) {
            ldk(ks + 1, a1, b1);
#pragma unroll
            for (int t = 0; t < 9; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0[t], acc[t], 0, 0, 0);
            if (ks + 2 < P / 2) ldk(ks + 2, a0, b0);
#pragma unroll
            for (int t = 0; t < 9; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1[t], acc[t], 0, 0, 0);
        }
        if (do_db) {
            float s = 0.f;
            for (int p = 0; p < P; ++p) s += dys[p * 64 + tid];
            dbacc += s;
        }
    }

    const int ci = ci0 + wn * 32 + (lane & 31);
    if (ci < a.Cin) {
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = co0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                a.part[((size_t)(split * 9 + t) * a.Cout + co) * a.Cin + ci] = acc[t][r];
            }
    }
    if (do_db) a.dbpart[(size_t)split * a.Cout + co0 + tid] = dbacc;
}

// ---------------------------------------------------------------------------
// Weight gradient for a narrow input (Cin <= 8: the RGB image padded to 8).
// GEMM M = 64 co, N = (tap, ci) = 72 columns (3 MFMA column blocks of 32, last
// partly padding), K = pixels.  3 waves, wave w owns column block w and both
// 32-row co blocks over all k-steps (no cross-wave reduction).  Same partial
// layout as the generic kernel, so the split-K reduce is shared.
// ---------------------------------------------------------------------------
template <int TH, int TW>
__global__ void __launch_bounds__(192) conv3x3_wgrad_c8_kernel(WgradArgs a) {
    constexpr int P = TH * TW, HWD = TW + 2, NHALO = (TH + 2) * HWD;
    constexpr int NT = 192;
    constexpr int DY_VEC = P * 16, X_VEC = NHALO * 2;
    constexpr int DY_PER = (DY_VEC + NT - 1) / NT, X_PER = (X_VEC + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) float smem[P * 64 + NHALO * 8];
    float* dys = smem;
    float* xs = smem + P * 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int NCO = a.Cout / 64;
    const int nb = blockIdx.x % NCO, split = blockIdx.x / NCO;
    const int co0 = nb * 64;
    const int t_begin = split * a.tps, t_end = min(a.ntiles, t_begin + a.tps);
    const int tpi = a.tiles_x * a.tiles_y;
    const int Cs = a.C0;  // <= 8

    // this lane's B column: j = 32*wave + (lane&31) -> (tap, ci); j >= 72 is padding
    const int j = 32 * wave + (lane & 31);
    const bool jvalid = j < 72;
    const int jt = jvalid ? j / 8 : 0, jc = j % 8;
    const int joff = ((jt / 3) * HWD + (jt % 3)) * 8 + jc;
    // this thread's 4 staged channels are fixed: (idx & 1) == (tid & 1)
    const Act4 xact = act_load4(a.sc0, a.sh0, (tid & 1) * 4);
    const bool xon = a.sc0 != nullptr;

    f32x4 rdy[DY_PER], rx[X_PER];
    unsigned xvalid = 0;
    auto gload = [&](int tile) {
        const int b = tile / tpi, trem = tile % tpi;
        const int ty0 = (trem / a.tiles_x) * TH, tx0 = (trem % a.tiles_x) * TW;
#pragma unroll
        for (int v = 0; v < DY_PER; ++v) {
            const int idx = tid + v * NT;
            f32x4 val = {0.f, 0.f, 0.f, 0.f};
            if (idx < DY_VEC) {
                const int p = idx >> 4, q = idx & 15;
                const int gy = ty0 + p / TW, gx = tx0 + p % TW;
                if (gy < a.H && gx < a.W)
                    val = *reinterpret_cast<const f32x4*>(
                        a.dy + ((size_t)(b * a.H + gy) * a.W + gx) * a.Cout + co0 + q * 4);
            }
            rdy[v] = val;
        }
        xvalid = 0;
#pragma unroll
        for (int v = 0; v < X_PER; ++v) {
            const int idx = tid + v * NT;
            f32x4 val = {0.f, 0.f, 0.f, 0.f};
            if (idx < X_VEC) {
                const int hp = idx >> 1, q = idx & 1;
                const int gy = ty0 - 1 + hp / HWD, gx = tx0 - 1 + hp % HWD;
                if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W && q * 4 < Cs) {
                    val = *reinterpret_cast<const f32x4*>(
                        a.src0 + ((size_t)(b * a.H + gy) * a.W + gx) * Cs + q * 4);
                    xvalid |= 1u << v;
                }
            }
            rx[v] = val;
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int v = 0; v < DY_PER; ++v) {
            const int idx = tid + v * NT;
            if (idx < DY_VEC) *reinterpret_cast<f32x4*>(&dys[idx * 4]) = rdy[v];
        }
#pragma unroll
        for (int v = 0; v < X_PER; ++v) {
            const int idx = tid + v * NT;
            if (idx < X_VEC) {
                f32x4 val = rx[v];
                if ((xvalid >> v) & 1u) val = act_reg4(val, xact, xon);
                *reinterpret_cast<f32x4*>(&xs[idx * 4]) = val;
            }
        }
    };

    f32x16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
    if (t_begin < t_end) gload(t_begin);
    for (int tile = t_begin; tile < t_end; ++tile) {
        __syncthreads();
        lstore();
        __syncthreads();
        if (tile + 1 < t_end) gload(tile + 1);
#pragma unroll 4
        for (int ks = 0; ks < P / 2; ++ks) {
            const int p = 2 * ks + (lane >> 5);
            const float a0 = dys[p * 64 + (lane & 31)];
            const float a1 = dys[p * 64 + 32 + (lane & 31)];
            const float bv = jvalid ? xs[((p / TW) * HWD + (p % TW)) * 8 + joff] : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv, acc1, 0, 0, 0);
        }
    }
    if (!jvalid || jc >= a.Cin) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        a.part[((size_t)(split * 9 + jt) * a.Cout + co) * a.Cin + jc] = acc0[r];
        a.part[((size_t)(split * 9 + jt) * a.Cout + co + 32) * a.Cin + jc] = acc1[r];
    }
}

// ---------------------------------------------------------------------------
// Image-layer weight gradient (inc.conv_op.0: the 3 real channels of the 8-channel
// padded image, no input activation, 64 outputs) on the fp32 VALU.  The GEMM is
// 64 x 27 x (B*H*W): through v_mfma_f32_32x32x2_f32 (conv3x3_wgrad_c8_kernel) it pads N
// 27 -> 96 and runs at the f32 MFMA rate, 219 us at bs16 x 256^2 for 301 MB of reads.
// Here a thread owns 2 output channels x all 27 (tap, ci) columns (54 accumulators)
// over an 8-pixel row segment: its dy (8 x float2; 32 lanes = one pixel's 64 channels,
// so loads are whole 256-B rows) times a sliding 10-value input row from a
// channel-planar LDS halo.  A persistent grid of WGI_GRID workgroups (8 waves) walks
// 4 x 32 tiles, prefetching the next tile's dy and halo into registers while the
// current one computes (about 100 VGPRs: 4 waves per SIMD); each workgroup then reduces
// its 16 segments (a lane shuffle, then a fixed 8 -> 4 -> 2 -> 1 wave tree in LDS) and
// writes one split-K partial slab (ci 3..7 as zeros) for wgrad_reduce_kernel.  The grid
// is a fixed count, so the summation order is device-independent.
// ---------------------------------------------------------------------------
#ifndef UGPG_WGI_GRID
#define UGPG_WGI_GRID 1024
#endif
constexpr int WGI_TH = 2, WGI_TW = 32, WGI_PX = 8, WGI_GRID = UGPG_WGI_GRID, WGI_NCI = 3;
// BN: dy formed from the following BatchNorm(+ReLU) backward while loading (a.bn_*: da, y
// and the apply's coefficients; bn_bwd_dy, bit-identical to the apply pass) -- the image
// layer's dy has no other reader (the input image needs no gradient), so the apply pass
// over the largest activation of the network is dropped
// TY: the storage of y (float, or __bf16: the bf16 arithmetic stores the image layer's output
// in bf16).  The next tile's (da, y) stay raw in registers while the current tile computes
// and dy is formed after it: forming dy at the fetch made every tile wait for its loads
// (the bf16-y form is held to 128 registers -- 2 workgroups per CU instead of 1, 8 B/lane of
// spills: 126 -> 99 us; the fp32-y form spills 48 B/lane there and is faster at 138)
template <bool BN, typename TY = float>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(std::is_same<TY, float>::value ? 1 : 4)))
conv3x3_wgrad_img_kernel(WgradArgs a) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    constexpr int TH = WGI_TH, TW = WGI_TW, PX = WGI_PX, NCI = WGI_NCI, CIN = 8, NT = 256;
    constexpr int HWP = TW + 4, HROWS = TH + 2, NH = HROWS * (TW + 2);
    constexpr int NACC = 2 * 9 * NCI;  // [c][ky][kx][ci]
    static_assert(NH <= NT, "one halo pixel per thread");
    __shared__ __attribute__((aligned(16))) float xs[2][NCI][HROWS * HWP];
    __shared__ float red[2][NACC][32];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tpi = a.tiles_x * a.tiles_y;
    // halo: one 4-channel piece (channels 0..3) per pixel, held channel-planar
    auto halo_fetch = [&](int tile) -> f32x4 {
        const int b = tile / tpi, trem = tile % tpi;
        const int ty0 = (trem / a.tiles_x) * TH, tx0 = (trem % a.tiles_x) * TW;
        const int gy = ty0 - 1 + tid / (TW + 2), gx = tx0 - 1 + tid % (TW + 2);
        f32x4 r = {0.f, 0.f, 0.f, 0.f};
        if (tile < a.ntiles && tid < NH && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)
            r = *reinterpret_cast<const f32x4*>(a.src0 + ((size_t)(b * a.H + gy) * a.W + gx) * CIN);
        return r;
    };
    auto halo_put = [&](int buf, f32x4 r) {
        if (tid < NH) {
            const int o = (tid / (TW + 2)) * HWP + tid % (TW + 2);
#pragma unroll
            for (int c = 0; c < NCI; ++c) xs[buf][c][o] = r[c];
        }
    };
    // thread: channels 2*cp, 2*cp+1 of the 8-pixel segment (row, c0..c0+7)
    const int cp = lane & 31, seg = tid >> 5, row = seg / (TW / PX), c0 = (seg % (TW / PX)) * PX;
    // BN: this thread's two channels' (scale, shift, mean, invstd, k0, k1)
    f2 bc[BN ? 6 : 1];
    if constexpr (BN) {
        const float* src[6] = {a.bn_scale, a.bn_shift, a.bn_mean, a.bn_invstd, a.bn_coef,
                               a.bn_coef + 64};
#pragma unroll
        for (int i = 0; i < 6; ++i) bc[i] = *reinterpret_cast<const f2*>(src[i] + 2 * cp);
    }
    // raw operands of one tile's dy: da (or dy) and y of this thread's 8 pixels x 2 channels
    // (pixels past the image / tiles past the end: zero dy, bit ok clear)
    typedef typename std::conditional<std::is_same<TY, float>::value, f2, uint32_t>::type yv_t;
    struct Raw {
        f2 g[PX];
        yv_t v[BN ? PX : 1];
        uint32_t ok;
    };
    auto dy_fetch = [&](int tile, Raw& r) {
        const int b = tile / tpi, trem = tile % tpi;
        const int gy = (trem / a.tiles_x) * TH + row, gx0 = (trem % a.tiles_x) * TW + c0;
        const size_t o = ((size_t)(b * a.H + gy) * a.W + gx0) * 64 + 2 * cp;
        r.ok = 0;
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            r.g[p] = f2{0.f, 0.f};
            if constexpr (BN) r.v[p] = yv_t{};
            if (tile < a.ntiles && gy < a.H && gx0 + p < a.W) {
                r.ok |= 1u << p;
                if constexpr (BN) {
                    r.g[p] = *reinterpret_cast<const f2*>(a.bn_da + o + (size_t)p * 64);
                    if constexpr (std::is_same<TY, float>::value)
                        r.v[p] = *reinterpret_cast<const f2*>(a.bn_y + o + (size_t)p * 64);
                    else
                        r.v[p] = *reinterpret_cast<const uint32_t*>(a.bn_y16 + o + (size_t)p * 64);
                } else {
                    r.g[p] = *reinterpret_cast<const f2*>(a.dy + o + (size_t)p * 64);
                }
            }
        }
    };
    auto dy_form = [&](const Raw& r, f2* d) {
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            if constexpr (BN) {
                f2 v;
                if constexpr (std::is_same<TY, float>::value) {
                    v = r.v[p];
                } else {  // exact widening of the two bf16
                    v = f2{__uint_as_float(r.v[p] << 16), __uint_as_float(r.v[p] & 0xffff0000u)};
                }
#pragma unroll
                for (int c = 0; c < 2; ++c)
                    d[p][c] = (r.ok >> p) & 1u ? bn_bwd_dy(r.g[p][c], v[c], bc[0][c], bc[1][c], bc[2][c],
                                                           bc[3][c], bc[4][c], bc[5][c])
                                               : 0.f;
            } else {
                d[p] = r.g[p];
            }
        }
    };
    float acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = 0.f;
    f2 d[PX];
    int buf = 0;
    if ((int)blockIdx.x < a.ntiles) {
        halo_put(0, halo_fetch(blockIdx.x));
        Raw r0;
        dy_fetch(blockIdx.x, r0);
        dy_form(r0, d);
    }
    __syncthreads();
    for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x, buf ^= 1) {
        // next tile (zeros past the end: no branch for the compiler to sink the FMAs past)
        const int nxt = tile + gridDim.x;
        const f32x4 hn = halo_fetch(nxt);
        Raw rn;
        dy_fetch(nxt, rn);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int ci = 0; ci < NCI; ++ci) {
                const float* xr = &xs[buf][ci][(row + ky) * HWP + c0];
                float x[PX + 2];
#pragma unroll
                for (int k = 0; k < PX / 4; ++k) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + 4 * k);
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[4 * k + i] = v[i];
                }
                const f2 xt = *reinterpret_cast<const f2*>(xr + PX);
                x[PX] = xt.x;
                x[PX + 1] = xt.y;
#pragma unroll
                for (int kx = 0; kx < 3; ++kx)
#pragma unroll
                    for (int p = 0; p < PX; ++p)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            float& r = acc[((c * 3 + ky) * 3 + kx) * NCI + ci];
                            r = fmaf(d[p][c], x[p + kx], r);
                        }
                // pin this row's products here: otherwise they are sunk below the halo store
                // and all 9 input rows are live at once (registers, hence occupancy)
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int kx = 0; kx < 3; ++kx) asm volatile("" : "+v"(acc[((c * 3 + ky) * 3 + kx) * NCI + ci]));
            }
        halo_put(buf ^ 1, hn);
        dy_form(rn, d);
        __syncthreads();
    }
    // the 2 segments of a wave that share cp (lane bit 5), then waves 4 -> 2 -> 1
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] += __shfl_xor(acc[i], 32, 64);
#pragma unroll
    for (int half = 2; half >= 1; half >>= 1) {
        if (wave >= half && wave < 2 * half && lane < 32)
#pragma unroll
            for (int i = 0; i < NACC; ++i) red[wave - half][i][cp] = acc[i];
        __syncthreads();
        if (wave < half && lane < 32)
#pragma unroll
            for (int i = 0; i < NACC; ++i) acc[i] += red[wave][i][cp];
        __syncthreads();
    }
    if (wave != 0 || lane >= 32) return;
    float* part = a.part + (size_t)blockIdx.x * 9 * 64 * CIN;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            float v[CIN];
#pragma unroll
            for (int ci = 0; ci < CIN; ++ci)
                v[ci] = ci < NCI ? acc[((c * 3 + t / 3) * 3 + t % 3) * NCI + ci] : 0.f;
            f32x4* o = reinterpret_cast<f32x4*>(part + ((size_t)t * 64 + 2 * cp + c) * CIN);
            o[0] = f32x4{v[0], v[1], v[2], v[3]};
            o[1] = f32x4{v[4], v[5], v[6], v[7]};
        }
}

// Fixed-order split-K reduction over the flat [9][Cout][Cin] partial slabs.
// Block = 64 consecutive slab elements (16 lanes x float4) x 16 split-groups;
// thread (g, l) sums splits g, g+16, ... in order, then a fixed 16-way LDS tree
// (deterministic: the summation order depends only on nsplit).
constexpr int WR_GROUPS = 16;
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* part, const float* dbpart,
                                                           int nsplit, int Cout, int Cin,
                                                           int Cin_real, float* dw, float* db,
                                                           int accumulate) {
    __shared__ f32x4 red[WR_GROUPS][16];
    const int l = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int64_t slab = (int64_t)9 * Cout * Cin;  // multiple of 4 (Cin % 4 == 0)
    const int64_t nvec = slab / 4;
    for (int64_t v0 = (int64_t)blockIdx.x * 16; v0 < nvec; v0 += (int64_t)gridDim.x * 16) {
        const int64_t v = v0 + l;
        f32x4 s = {0.f, 0.f, 0.f, 0.f};
        if (v < nvec) {
            const f32x4* p = reinterpret_cast<const f32x4*>(part) + v;
            int k = grp;
            for (; k + 3 * WR_GROUPS < nsplit; k += 4 * WR_GROUPS) {
                const f32x4 a0 = p[(size_t)k * nvec], a1 = p[(size_t)(k + WR_GROUPS) * nvec];
                const f32x4 a2 = p[(size_t)(k + 2 * WR_GROUPS) * nvec];
                const f32x4 a3 = p[(size_t)(k + 3 * WR_GROUPS) * nvec];
                s += a0;
                s += a1;
                s += a2;
                s += a3;
            }
            for (; k < nsplit; k += WR_GROUPS) s += p[(size_t)k * nvec];
        }
        red[grp][l] = s;
        __syncthreads();
        if (threadIdx.x < 64) {
            // 64 threads: element e = 4*l' + j of this block's 64-element run
            const int lv = threadIdx.x >> 2, j = threadIdx.x & 3;
            float acc = 0.f;
#pragma unroll
            for (int g = 0; g < WR_GROUPS; ++g) acc += red[g][lv][j];
            const int64_t e = (v0 + lv) * 4 + j;
            if (v0 + lv < nvec) {
                const int ci = (int)(e % Cin);
                const int64_t r = e / Cin;
                const int co = (int)(r % Cout), t = (int)(r / Cout);
                if (ci < Cin_real) {
                    const size_t o = ((size_t)co * Cin_real + ci) * 9 + t;
                    dw[o] = accumulate ? dw[o] + acc : acc;
                }
            }
        }
        __syncthreads();
    }
    if (db && blockIdx.x == 0) {
        for (int co = threadIdx.x; co < Cout; co += blockDim.x) {
            float s = 0.f;
            for (int k = 0; k < nsplit; ++k) s += dbpart[(size_t)k * Cout + co];
            db[co] = accumulate ? db[co] + s : s;
        }
    }
}

// The same reduction for few splits (<= 16: the wide-channel layers, large slabs), each
// (element, tap) summed over the splits in order, written as contiguous OIHW runs
// (wgrad_reduce_kernel's writes there are 4 B at a 36-B stride, each line assembled by
// blocks on different XCDs).
// Block = 64 consecutive element quads x the 9 taps (wave t = tap t: coalesced reads of one
// tap plane); the quads' 9-tap sums meet in LDS and leave as the block's 2304 contiguous OIHW
// floats (one f32x4 per thread).  (A thread per quad with all 9 taps -- 4 waves per CU at
// 512 x 512 -- ran at 3.4 TB/s.)
__global__ void __launch_bounds__(576) wgrad_reduce_few_kernel(const float* part, int nsplit,
                                                               int Cout, int Cin, float* dw,
                                                               int accumulate) {
    __shared__ f32x4 sm[64][9];
    const int l = threadIdx.x & 63, t = threadIdx.x >> 6;
    const int64_t n4 = (int64_t)Cout * Cin / 4, m4 = (int64_t)blockIdx.x * 64 + l;
    if (m4 < n4) {
        const f32x4* p = reinterpret_cast<const f32x4*>(part) + (size_t)t * n4 + m4;
        // every split's load in flight, then the sum in split order (nsplit <= 16)
        f32x4 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (k < nsplit) v[k] = p[(size_t)k * 9 * n4];
        f32x4 s = v[0];
#pragma unroll
        for (int k = 1; k < 16; ++k)
            if (k < nsplit) s += v[k];
        sm[l][t] = s;
    }
    __syncthreads();
    // element e = 4*m4 + j, tap t -> dw[e*9 + t]: the block's 64 quads are 2304 floats
    const int64_t f0 = (int64_t)blockIdx.x * 64 * 36, nf = n4 * 36;
    const int i = threadIdx.x;  // f32x4 i of the block's run
    if (f0 + 4 * i < nf) {
        f32x4 r;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int f = 4 * i + u, e = f / 9, tt = f % 9;
            r[u] = sm[e >> 2][tt][e & 3];
        }
        f32x4* o = reinterpret_cast<f32x4*>(dw + f0) + i;
        if (accumulate) r += *o;
        *o = r;
    }
}

__global__ void pack_conv3x3_kernel(const float* w, float* wpk, int Cout, int Cin, int Cin_pad,
                                    int mode) {
    // mode 0: wpk[Cin_pad/8][9][Cout][8];  mode 1: wpk[Cout/8][9][Cin_pad][8] (rot180, transposed)
    const int64_t total = (int64_t)Cin_pad * 9 * Cout;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(e & 7);
        int64_t r = e >> 3;
        if (mode == 0) {
            const int co = (int)(r % Cout);
            r /= Cout;
            const int t = (int)(r % 9), cg = (int)(r / 9);
            const int ci = cg * 8 + j;
            wpk[e] = ci < Cin ? w[((size_t)co * Cin + ci) * 9 + t] : 0.f;
        } else {
            const int ci = (int)(r % Cin_pad);
            r /= Cin_pad;
            const int t = (int)(r % 9), cg = (int)(r / 9);
            const int co = cg * 8 + j;
            wpk[e] = ci < Cin ? w[((size_t)co * Cin + ci) * 9 + (8 - t)] : 0.f;
        }
    }
}

// ---------------------------------------------------------------------------
// host-side configuration
// ---------------------------------------------------------------------------
namespace {

// (A CFG_W variant register-capped to 3 waves/SIMD spills 7 VGPRs and measured
// 5-30% slower on every layer: 2 blocks/CU it is.)
enum FwdCfg { CFG_L = 0, CFG_W = 1, CFG_S = 2, NUM_CFG = 3 };
struct FwdShape {
    int th, tw, bn;
};
const FwdShape kFwd[NUM_CFG] = {{16, 16, 64}, {8, 16, 128}, {8, 8, 64}};

int64_t fwd_blocks(int cfg, int B, int H, int W, int Cout) {
    const FwdShape& s = kFwd[cfg];
    return (int64_t)B * cdiv(H, s.th) * cdiv(W, s.tw) * (Cout / s.bn);
}

int pick_fwd_cfg(int B, int H, int W, int Cout, int split) {
    // prefer the larger tiles while they still give >= 2 blocks per CU; a block
    // must not straddle the output split (its BN must divide `split`)
    const int64_t want = 512;
    if (Cout % 128 == 0 && split % 128 == 0 && fwd_blocks(CFG_W, B, H, W, Cout) >= want)
        return CFG_W;
    if (fwd_blocks(CFG_L, B, H, W, Cout) >= want) return CFG_L;
    return CFG_S;
}

constexpr int WG_TH = 4, WG_TW = 16;

struct WgradPlan {
    int tiles_x, tiles_y, ntiles, nsplit, tps;
};

WgradPlan wgrad_plan(int B, int H, int W, int Cin, int Cout, int th = WG_TH, int tw = WG_TW) {
    WgradPlan p;
    p.tiles_x = (int)cdiv(W, tw);
    p.tiles_y = (int)cdiv(H, th);
    p.ntiles = B * p.tiles_x * p.tiles_y;
    const int64_t base = (int64_t)(Cout / 64) * cdiv(Cin, 64);
    // 2 co-resident blocks per CU (232 VGPR+AGPR, 44 KB LDS): aim for a multiple of 512
    int64_t ns = cdiv(512, base);
    if (ns * base < 512) ns = cdiv(1024, base);
    // cap the fp32 partial slab at 192 MB
    const int64_t per = (int64_t)9 * Cout * Cin * 4;
    int64_t cap = (192ll << 20) / per;
    if (cap < 1) cap = 1;
    if (ns > cap) ns = cap;
    if (ns > p.ntiles) ns = p.ntiles;
    if (ns < 1) ns = 1;
    p.tps = (int)cdiv(p.ntiles, ns);
    p.nsplit = (int)cdiv(p.ntiles, p.tps);
    return p;
}

// Narrow-input wgrad (conv3x3_wgrad_c8_kernel): 8x16-pixel tiles, 4 blocks/CU by
// LDS (38.5 KB) -> aim for 1024 blocks.
constexpr int WG8_TH = 8, WG8_TW = 16;

static bool wgrad_use_c8(int C0, int C1, const void* db) { return C1 == 0 && C0 <= 8 && !db; }

WgradPlan wgrad_plan_c8(int B, int H, int W, int Cout) {
    WgradPlan p;
    p.tiles_x = (int)cdiv(W, WG8_TW);
    p.tiles_y = (int)cdiv(H, WG8_TH);
    p.ntiles = B * p.tiles_x * p.tiles_y;
    int64_t ns = cdiv(1024, Cout / 64);
    if (ns > p.ntiles) ns = p.ntiles;
    if (ns < 1) ns = 1;
    p.tps = (int)cdiv(p.ntiles, ns);
    p.nsplit = (int)cdiv(p.ntiles, p.tps);
    return p;
}

template <int TH, int TW, int BN, int BKC, int WM, int WN, int MINW = 1>
void launch_fwd(const ConvFwdArgs& a, hipStream_t st) {
    const unsigned grid = (unsigned)((int64_t)a.ntiles * (a.Cout / BN));
    hipLaunchKernelGGL((conv3x3_fwd_kernel<TH, TW, BN, BKC, WM, WN, MINW>), dim3(grid), dim3(256),
                       0, st, a);
}

}  // namespace
}  // namespace ugpg

using namespace ugpg;

extern "C" int ugpg_conv3x3_fwd_ntiles(int B, int H, int W, int Cin, int Cout, int wfmt) {
    if (wfmt == UGPG_WFMT_X6 || wfmt == UGPG_WFMT_BF16) {
        const int np = wfmt == UGPG_WFMT_X6 ? 3 : 1;
        return fwd_x6_stat_slots(x6_fwd_form(B, H, W, Cin, Cout, np), B, H, W);
    }
    if (img_fwd_eligible(W, Cin, 0, Cout)) return img_fwd_slots(B, H, W, 2);
    const int cfg = pick_fwd_cfg(B, H, W, Cout, Cout);
    return (int)(B * cdiv(H, kFwd[cfg].th) * cdiv(W, kFwd[cfg].tw));
}

extern "C" int ugpg_conv3x3_fwd(const ugpg_conv_t* p, void* stream) {
    if (!p || (!p->src[0].data && !p->src[0].data_bf16) || !p->wpk ||
        (!p->out[0] && !p->out_bf16)) {
        set_error("conv3x3_fwd: null argument");
        return UGPG_ERR_INVALID;
    }
    const bool has1 = p->src[1].data || p->src[1].data_bf16;
    const int C0 = p->src[0].C, C1 = has1 ? p->src[1].C : 0;
    const int Cin = C0 + C1;
    if (Cin % 8 || C0 % 8 || p->Cout % 64 || p->B <= 0 || p->H <= 0 || p->W <= 0) {
        set_error("conv3x3_fwd: unsupported shape Cin=%d (C0=%d) Cout=%d", Cin, C0, p->Cout);
        return UGPG_ERR_INVALID;
    }
    if (p->out_split <= 0 || p->out_split > p->Cout || p->out_split % 64 ||
        (p->out_split < p->Cout && !p->out[1])) {
        set_error("conv3x3_fwd: bad out_split %d (Cout %d)", p->out_split, p->Cout);
        return UGPG_ERR_INVALID;
    }
    const bool split = p->wfmt == UGPG_WFMT_X6 || p->wfmt == UGPG_WFMT_BF16;
    if (p->wfmt != UGPG_WFMT_F32 && !split) {
        set_error("conv3x3_fwd: unknown weight format %d", p->wfmt);
        return UGPG_ERR_INVALID;
    }
    // an 8-channel single source (the padded image) is zero-extended to one 16-channel
    // chunk: the weights must then be packed with K = 16 (ugpg_pack_conv3x3 cin_pad 16)
    const bool ext8 = split && C0 == 8 && C1 == 0;
    if (split && !ext8 && (C0 % 16 || C1 % 16)) {
        set_error("conv3x3_fwd: split-bf16 path needs 16-channel sources (C0=%d C1=%d)", C0, C1);
        return UGPG_ERR_INVALID;
    }
    // bf16 activation storage (data / out[0] NULL): the single-piece persistent form reads
    // and writes it (images >= 32 wide); the image-layer kernel writes it
    const bool b16_in = !p->src[0].data || (has1 && !p->src[1].data);
    const bool b16_out = !p->out[0];
    const bool x6r_np1 = p->wfmt == UGPG_WFMT_BF16 && p->W >= 32;
    const bool img = p->wfmt == UGPG_WFMT_F32 && img_fwd_eligible(p->W, C0, C1, p->Cout);
    if ((b16_in && !x6r_np1) || (b16_out && !(x6r_np1 || img)) ||
        (b16_out && (p->out_split != p->Cout || p->accumulate[0]))) {
        set_error("conv3x3_fwd: bf16-only activations (src data / out[0] NULL) need the bf16 "
                  "weight format and an image >= 32 wide (or, for the output, the fp32 image "
                  "layer), one output and no accumulate");
        return UGPG_ERR_INVALID;
    }
    const bool bnb = p->bnb_part != nullptr;
    if (bnb && ((!p->bnb_y && !p->bnb_y_bf16) || !p->bnb_mean || !p->bnb_invstd || !p->bnb_scale || !p->bnb_shift ||
                p->out_split != p->Cout || p->accumulate[0] || p->Cout > 1024)) {
        set_error("conv3x3_fwd: BatchNorm-backward partials need bnb_y/mean/invstd/scale/shift, "
                  "one output and no accumulate");
        return UGPG_ERR_INVALID;
    }
    if (bnb && b16_out && !p->bnb_y_bf16) {
        set_error("conv3x3_fwd: a bf16-only output with BatchNorm-backward partials needs the "
                  "BN input in bf16 (bnb_y_bf16)");
        return UGPG_ERR_INVALID;
    }
    if (p->stats && (p->out_split != p->Cout || p->accumulate[0])) {
        set_error("conv3x3_fwd: BatchNorm partials (stats) need one output and no accumulate");
        return UGPG_ERR_INVALID;
    }
    // the caller's partial buffers must hold every slot the launched form writes (the
    // form, hence the slot count, is a function of the shape and wfmt only)
    if (p->stats || bnb) {
        const int need = ugpg_conv3x3_fwd_ntiles(p->B, p->H, p->W, Cin, p->Cout, p->wfmt);
        if (p->stats && p->stats_slots < need) {
            set_error("conv3x3_fwd: stats holds %d slots, this call writes %d", p->stats_slots,
                      need);
            return UGPG_ERR_WORKSPACE;
        }
        if (bnb && p->bnb_slots < need) {
            set_error("conv3x3_fwd: bnb_part holds %d slots, this call writes %d", p->bnb_slots,
                      need);
            return UGPG_ERR_WORKSPACE;
        }
    }
    ConvFwdArgs a;
    a.bnb_y = yref(p->bnb_y, p->bnb_y_bf16);
    a.bnb_mean = p->bnb_mean;
    a.bnb_invstd = p->bnb_invstd;
    a.bnb_scale = p->bnb_scale;
    a.bnb_shift = p->bnb_shift;
    a.bnb_part = p->bnb_part;
    a.src0_16 = static_cast<const __bf16*>(p->src[0].data_bf16);
    a.src1_16 = has1 ? static_cast<const __bf16*>(p->src[1].data_bf16) : nullptr;
    a.out0_16 = static_cast<__bf16*>(p->out_bf16);
    if (p->out_bf16 && (p->out_split != p->Cout || p->accumulate[0])) {
        set_error("conv3x3_fwd: out_bf16 needs one output without accumulate");
        return UGPG_ERR_INVALID;
    }
    // forms that do not write the bf16 copy themselves: a cast pass after the conv
    auto out16_pass = [&]() {
        return ugpg_cast_f32_bf16(p->out[0], static_cast<uint16_t*>(p->out_bf16),
                                  (int64_t)p->B * p->H * p->W * p->Cout, stream);
    };
    // forms that do not fuse the partials: the same reduction as a pass after the conv
    auto bnb_pass = [&]() {
        const int nslots = ugpg_conv3x3_fwd_ntiles(p->B, p->H, p->W, Cin, p->Cout, p->wfmt);
        launch_bn_bwd_reduce(p->out[0], a.bnb_y, (int64_t)p->B * p->H * p->W, p->Cout,
                             p->bnb_mean, p->bnb_invstd, p->bnb_scale, p->bnb_shift, p->bnb_part,
                             nslots, as_stream(stream));
    };
    a.src0 = p->src[0].data;
    a.sc0 = p->src[0].scale;
    a.sh0 = p->src[0].shift;
    a.C0 = C0;
    a.src1 = p->src[1].data;
    a.sc1 = p->src[1].scale;
    a.sh1 = p->src[1].shift;
    a.C1 = C1;
    a.wpk = p->wpk;
    a.bias = p->bias;
    a.out0 = p->out[0];
    a.out1 = p->out[1];
    a.split = p->out_split;
    a.acc0 = p->accumulate[0];
    a.acc1 = p->accumulate[1];
    a.stats = p->stats;
    a.B = p->B;
    a.H = p->H;
    a.W = p->W;
    a.Cin = ext8 ? 16 : Cin;
    a.Cout = p->Cout;
    hipStream_t st = as_stream(stream);
    if (split) {
        const int np = p->wfmt == UGPG_WFMT_X6 ? 3 : 1;
        if (np == 1 && p->W >= 16 && C0 + C1 > 2048) {  // X6R_CTAB_MAX (conv_x6.hip)
            set_error("conv3x3_fwd: the bf16 persistent form takes at most 2048 input channels");
            return UGPG_ERR_INVALID;
        }
        const X6Form f = x6_fwd_form(p->B, p->H, p->W, Cin, p->Cout, np);
        a.tiles_x = (int)cdiv(p->W, f.tw);
        a.tiles_y = (int)cdiv(p->H, f.th);
        a.ntiles = p->B * a.tiles_x * a.tiles_y;
        const int wrote = launch_fwd_x6(a, np, st);
        if (bnb && !(wrote & FWD_WROTE_BNB)) bnb_pass();
        if (int e = check_launch("conv3x3_fwd_x6")) return e;
        return p->out_bf16 && !(wrote & FWD_WROTE_OUT16) ? out16_pass() : UGPG_OK;
    }
    if (img_fwd_eligible(p->W, C0, C1, p->Cout)) {
        // the image layer in fp32 / bf16 mode: the direct fp32 kernel on the fp32 pack
        a.tiles_x = (int)cdiv(p->W, 32);
        a.tiles_y = (int)cdiv(p->H, 8);
        a.ntiles = p->B * a.tiles_x * a.tiles_y;
        if (launch_img_fwd(a, true, st)) return check_launch("conv3x3_img_fwd");  // + out16
        if (p->stats || b16_out) {  // ugpg_conv3x3_fwd_ntiles counted the image kernel's slots
            set_error("conv3x3_fwd: BatchNorm partials of an 8-channel source need one "
                      "output without accumulate");
            return UGPG_ERR_INVALID;
        }
    }
    const int cfg = pick_fwd_cfg(p->B, p->H, p->W, p->Cout, p->out_split);
    if (p->out_split % kFwd[cfg].bn) {
        set_error("conv3x3_fwd: out_split %d not a multiple of the tile width %d", p->out_split,
                  kFwd[cfg].bn);
        return UGPG_ERR_INVALID;
    }
    const bool bk16 = (C0 % 16 == 0) && (C1 % 16 == 0);
    const FwdShape& s = kFwd[cfg];
    a.tiles_x = (int)cdiv(p->W, s.tw);
    a.tiles_y = (int)cdiv(p->H, s.th);
    a.ntiles = p->B * a.tiles_x * a.tiles_y;
    switch (cfg) {
        case CFG_L:
            if (bk16) launch_fwd<16, 16, 64, 16, 4, 1>(a, st);
            else launch_fwd<16, 16, 64, 8, 4, 1>(a, st);
            break;
        case CFG_W:
            launch_fwd<8, 16, 128, 8, 2, 2>(a, st);
            break;
        default:
            if (bk16) launch_fwd<8, 8, 64, 16, 2, 2>(a, st);
            else launch_fwd<8, 8, 64, 8, 2, 2>(a, st);
            break;
    }
    if (bnb) bnb_pass();
    if (int e = check_launch("conv3x3_fwd")) return e;
    return p->out_bf16 ? out16_pass() : UGPG_OK;
}

extern "C" size_t ugpg_pack_conv3x3_bytes(int Cout, int Cin_pad, int wfmt) {
    const size_t n = (size_t)Cin_pad * 9 * Cout;
    return wfmt == UGPG_WFMT_X6 ? n * 3 * 2 : wfmt == UGPG_WFMT_BF16 ? n * 2 : n * 4;
}

extern "C" int ugpg_pack_conv3x3(const float* w, void* wpk, int Cout, int Cin, int Cin_pad,
                                 int mode, int wfmt, void* stream) {
    if (!w || !wpk || Cin_pad < Cin || Cin_pad % 8 || (mode == 1 && Cout % 8) || mode < 0 ||
        mode > 1 || (wfmt != UGPG_WFMT_F32 && wfmt != UGPG_WFMT_X6 && wfmt != UGPG_WFMT_BF16)) {
        set_error("pack_conv3x3: bad arguments (Cout=%d Cin=%d Cin_pad=%d mode=%d wfmt=%d)", Cout,
                  Cin, Cin_pad, mode, wfmt);
        return UGPG_ERR_INVALID;
    }
    if (wfmt == UGPG_WFMT_X6 || wfmt == UGPG_WFMT_BF16) {
        const int N = mode == 0 ? Cout : Cin_pad, K = mode == 0 ? Cin_pad : Cout;
        if (N % 64 || K % 16) {
            set_error("pack_conv3x3: split-bf16 format needs N %% 64 == 0 and K %% 16 == 0 "
                      "(N=%d K=%d)", N, K);
            return UGPG_ERR_INVALID;
        }
        launch_pack_x6(w, wpk, Cout, Cin, Cin_pad, mode, wfmt == UGPG_WFMT_X6 ? 3 : 1,
                       as_stream(stream));
        return check_launch("pack_conv3x3_x6");
    }
    const int64_t total = (int64_t)Cin_pad * 9 * Cout;
    hipLaunchKernelGGL(pack_conv3x3_kernel, dim3(stream_grid(total)), dim3(256), 0,
                       as_stream(stream), w, static_cast<float*>(wpk), Cout, Cin, Cin_pad, mode);
    return check_launch("pack_conv3x3");
}

extern "C" int ugpg_pack_conv3x3_batch(const ugpg_pack_item_t* items, int n, int wfmt,
                                       void* stream) {
    if (!items || n < 0 || (wfmt != UGPG_WFMT_X6 && wfmt != UGPG_WFMT_BF16)) {
        set_error("pack_conv3x3_batch: bad arguments (n=%d wfmt=%d)", n, wfmt);
        return UGPG_ERR_INVALID;
    }
    std::vector<PackItem> v((size_t)n);
    for (int i = 0; i < n; ++i) {
        const ugpg_pack_item_t& q = items[i];
        const int N = q.mode == 0 ? q.Cout : q.Cin_pad, K = q.mode == 0 ? q.Cin_pad : q.Cout;
        if (!q.w || !q.wpk || q.Cin_pad < q.Cin || q.Cin_pad % 8 || q.mode < 0 || q.mode > 1 ||
            (q.mode == 1 && q.Cout % 8) || N % 64 || K % 16) {
            set_error("pack_conv3x3_batch: bad item %d (Cout=%d Cin=%d Cin_pad=%d mode=%d)", i,
                      q.Cout, q.Cin, q.Cin_pad, q.mode);
            return UGPG_ERR_INVALID;
        }
        v[i] = PackItem{q.w, q.wpk, q.Cout, q.Cin, q.Cin_pad, q.mode};
    }
    if (n == 0) return UGPG_OK;
    launch_pack_x6_batch(v.data(), n, wfmt == UGPG_WFMT_X6 ? 3 : 1, as_stream(stream));
    return check_launch("pack_conv3x3_batch");
}

static int wgrad_c1(const ugpg_wgrad_t* p) {
    return p->src[1].data || p->src[1].data_bf16 ? p->src[1].C : 0;
}
// bf16 activation storage of the sources (data NULL): all sources alike
static bool wgrad_b16(const ugpg_wgrad_t* p) { return !p->src[0].data; }

static int wgrad_check(const ugpg_wgrad_t* p) {
    if (!p || (!p->src[0].data && !p->src[0].data_bf16) ||
        (!p->dy && !p->dy_bf16 && !p->dy_bn) || !p->dw) {
        set_error("conv3x3_wgrad: null argument");
        return UGPG_ERR_INVALID;
    }
    const int C0 = p->src[0].C, C1 = wgrad_c1(p);
    if (const ugpg_bn_lazy_t* l = p->dy_bn) {  // dy formed while loading
        // the image layer's kernel (8-channel image, no activation, 64 outputs: wgrad_kind's
        // WG_IMG) forms it too, with no other reader of dy (dy_out == NULL)
        const bool img = C1 == 0 && C0 == 8 && !p->db && !p->src[0].scale && p->Cout == 64 &&
                         p->Cin_real > 0 && p->Cin_real <= WGI_NCI && !p->dy && !p->dy_bf16 &&
                         !wgrad_b16(p) && l->da && !l->y != !l->y_bf16 && l->mean && l->invstd && l->scale &&
                         l->shift && l->coef && !l->dy_out && !l->route_src && !l->route_argmax;
        if (img) return UGPG_OK;
        if (p->dy || p->dy_bf16 || p->math != UGPG_WFMT_X6 || p->db || C0 % 64 || C1 % 64 ||
            wgrad_b16(p) || p->Cout % 64 || p->Cin_real > C0 + C1 ||
            (!l->da && !l->route_src) || !l->route_src != !l->route_argmax || !l->y || l->y_bf16 ||
            !l->mean || !l->invstd || !l->scale || !l->shift || !l->coef ||
            (l->dy_out && (l->dy_out == l->da || l->dy_out == l->y))) {
            set_error("conv3x3_wgrad: dy_bn needs the split-bf16 arithmetic, fp32 sources of "
                      "64-channel multiples, no dy, no bias gradient and every BatchNorm input "
                      "(C0=%d C1=%d Cout=%d)", C0, C1, p->Cout);
            return UGPG_ERR_INVALID;
        }
        return UGPG_OK;
    }
    if (!p->dy && (p->math != UGPG_WFMT_BF16 || p->db || C0 % 64 || C1 % 64)) {
        set_error("conv3x3_wgrad: a bf16-stored dy needs the bf16 arithmetic, 64-channel "
                  "sources and no bias gradient");
        return UGPG_ERR_INVALID;
    }
    if (wgrad_b16(p) != (C1 && !p->src[1].data) && C1) {
        set_error("conv3x3_wgrad: both sources must be stored alike (fp32 or bf16)");
        return UGPG_ERR_INVALID;
    }
    if (wgrad_b16(p) && (p->math != UGPG_WFMT_BF16 || p->db || C0 % 64 || C1 % 64)) {
        set_error("conv3x3_wgrad: bf16-stored sources need the bf16 arithmetic, 64-channel "
                  "sources and no bias gradient");
        return UGPG_ERR_INVALID;
    }
    if (p->Cout % 64 || C0 % 4 || (C1 && (C0 % 64 || C1 % 64)) || p->Cin_real > C0 + C1) {
        set_error("conv3x3_wgrad: unsupported shape C0=%d C1=%d Cout=%d", C0, C1, p->Cout);
        return UGPG_ERR_INVALID;
    }
    return UGPG_OK;
}

enum WgradKind { WG_GENERIC, WG_C8, WG_X6, WG_IMG };

static WgradKind wgrad_kind(const ugpg_wgrad_t* p, int C0, int C1) {
    if (C1 == 0 && C0 == 8 && !p->db && !p->src[0].scale && p->Cout == 64 &&
        p->Cin_real > 0 && p->Cin_real <= WGI_NCI)
        return WG_IMG;
    if (wgrad_use_c8(C0, C1, p->db)) return WG_C8;
    if ((p->math == UGPG_WFMT_X6 || p->math == UGPG_WFMT_BF16) && !p->db && C0 % 64 == 0 &&
        C1 % 64 == 0)
        return WG_X6;
    return WG_GENERIC;
}

static WgradPlan wgrad_plan_for(const ugpg_wgrad_t* p, WgradKind k, int Cin) {
    if (k == WG_C8) return wgrad_plan_c8(p->B, p->H, p->W, p->Cout);
    if (k == WG_IMG) {
        WgradPlan w;
        w.tiles_x = (int)cdiv(p->W, WGI_TW);
        w.tiles_y = (int)cdiv(p->H, WGI_TH);
        w.ntiles = p->B * w.tiles_x * w.tiles_y;
        w.nsplit = std::min(w.ntiles, WGI_GRID);  // one partial slab per workgroup
        w.tps = (int)cdiv(w.ntiles, w.nsplit);
        return w;
    }
    if (k == WG_X6) {
        WgradPlan w = wgrad_plan(p->B, p->H, p->W, Cin, p->Cout, WGX6W_TH, WGX6_TW);
        // persistent kernel: about one item per CU, planned for the MI355X's 256 CUs
        // (a fixed count keeps the split, hence the summation order, device-independent)
        wgrad_x6w_plan(w.ntiles, p->Cout, Cin, 256, w.nsplit, w.tps);
        return w;
    }
    return wgrad_plan(p->B, p->H, p->W, Cin, p->Cout);
}

extern "C" size_t ugpg_conv3x3_wgrad_workspace(const ugpg_wgrad_t* p) {
    if (wgrad_check(p)) return 0;
    const int C0 = p->src[0].C, C1 = wgrad_c1(p);
    const int Cin = C0 + C1;
    WgradPlan w = wgrad_plan_for(p, wgrad_kind(p, C0, C1), Cin);
    return ((size_t)w.nsplit * 9 * p->Cout * Cin + (size_t)w.nsplit * p->Cout) * sizeof(float);
}

extern "C" int ugpg_conv3x3_wgrad(const ugpg_wgrad_t* p, void* ws, size_t ws_bytes,
                                  void* stream) {
    if (int e = wgrad_check(p)) return e;
    const int C0 = p->src[0].C, C1 = wgrad_c1(p);
    const int Cin = C0 + C1;
    const WgradKind kind = wgrad_kind(p, C0, C1);
    WgradPlan w = wgrad_plan_for(p, kind, Cin);
    const size_t need = ugpg_conv3x3_wgrad_workspace(p);
    if (!ws || ws_bytes < need) {
        set_error("conv3x3_wgrad: workspace %zu < %zu", ws_bytes, need);
        return UGPG_ERR_WORKSPACE;
    }
    WgradArgs a;
    a.src0 = p->src[0].data;
    a.sc0 = p->src[0].scale;
    a.sh0 = p->src[0].shift;
    a.C0 = C0;
    a.src1 = p->src[1].data;
    a.sc1 = p->src[1].scale;
    a.sh1 = p->src[1].shift;
    a.C1 = C1;
    a.src0_16 = static_cast<const __bf16*>(p->src[0].data_bf16);
    a.src1_16 = static_cast<const __bf16*>(p->src[1].data_bf16);
    a.dy = p->dy;
    a.dy16 = p->dy ? nullptr : static_cast<const __bf16*>(p->dy_bf16);
    const ugpg_bn_lazy_t* bl = p->dy_bn;
    a.bn_da = bl ? bl->da : nullptr;
    a.bn_y = bl ? bl->y : nullptr;
    a.bn_mean = bl ? bl->mean : nullptr;
    a.bn_invstd = bl ? bl->invstd : nullptr;
    a.bn_scale = bl ? bl->scale : nullptr;
    a.bn_shift = bl ? bl->shift : nullptr;
    a.bn_coef = bl ? bl->coef : nullptr;
    a.bn_dy_out = bl ? bl->dy_out : nullptr;
    a.bn_rsrc = bl ? bl->route_src : nullptr;
    a.bn_ram = bl ? bl->route_argmax : nullptr;
    a.bn_y16 = bl ? static_cast<const __bf16*>(bl->y_bf16) : nullptr;
    a.Cout = p->Cout;
    a.Cin = Cin;
    a.part = static_cast<float*>(ws);
    a.dbpart = p->db ? a.part + (size_t)w.nsplit * 9 * p->Cout * Cin : nullptr;
    a.B = p->B;
    a.H = p->H;
    a.W = p->W;
    a.tiles_x = w.tiles_x;
    a.tiles_y = w.tiles_y;
    a.ntiles = w.ntiles;
    a.nsplit = w.nsplit;
    a.tps = w.tps;
    hipStream_t st = as_stream(stream);
    if (kind == WG_X6) {
        launch_wgrad_x6(a, p->math == UGPG_WFMT_BF16 ? 1 : 3, st);
    } else if (kind == WG_IMG) {
        if (a.bn_y)
            hipLaunchKernelGGL((conv3x3_wgrad_img_kernel<true, float>), dim3((unsigned)w.nsplit), dim3(256), 0, st, a);
        else if (a.bn_y16)
            hipLaunchKernelGGL((conv3x3_wgrad_img_kernel<true, __bf16>), dim3((unsigned)w.nsplit), dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL(conv3x3_wgrad_img_kernel<false>, dim3((unsigned)w.nsplit), dim3(256), 0, st, a);
    } else if (kind == WG_C8) {
        const unsigned grid = (unsigned)((p->Cout / 64) * w.nsplit);
        hipLaunchKernelGGL((conv3x3_wgrad_c8_kernel<WG8_TH, WG8_TW>), dim3(grid), dim3(192), 0, st,
                           a);
    } else {
        const unsigned grid = (unsigned)((p->Cout / 64) * cdiv(Cin, 64) * w.nsplit);
        hipLaunchKernelGGL((conv3x3_wgrad_kernel<WG_TH, WG_TW>), dim3(grid), dim3(256), 0, st, a);
    }
    if (int e = check_launch("conv3x3_wgrad")) return e;
    const int Cr = p->Cin_real > 0 ? p->Cin_real : Cin;
    if (w.nsplit <= 16 && Cr == Cin && !p->db && ((int64_t)p->Cout * Cin) % 4 == 0 &&
        reinterpret_cast<uintptr_t>(p->dw) % 16 == 0) {  // (dw may be a view of a flat buffer)
        const int64_t n4 = (int64_t)p->Cout * Cin / 4;
        hipLaunchKernelGGL(wgrad_reduce_few_kernel, dim3((unsigned)cdiv(n4, 64)), dim3(576), 0, st,
                           a.part, w.nsplit, p->Cout, Cin, p->dw, p->accumulate);
        return check_launch("conv3x3_wgrad_reduce");
    }
    int64_t rblocks = cdiv((int64_t)9 * p->Cout * Cin / 4, 16);
    if (rblocks > 4096) rblocks = 4096;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)rblocks), dim3(256), 0, st, a.part,
                       a.dbpart, w.nsplit, p->Cout, Cin, Cr, p->dw, p->db, p->accumulate);
    return check_launch("conv3x3_wgrad_reduce");
}
