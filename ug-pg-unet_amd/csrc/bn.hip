// BatchNorm2d(train/eval) + ReLU for NHWC fp32 on gfx950.
// Replaces aten::native_batch_norm / native_batch_norm_backward / threshold_backward
// behind DoubleConv (reference UG_unet_parts.py:11-12,14-15).
//
// Forward statistics come from the producing conv's epilogue as per-tile
// (count, sum, M2); ugpg_bn_finalize merges them in fp64 (Chan et al.), which is
// the numerically stable two-pass result, deterministic for a fixed tiling.
// The normalisation itself is never materialised: consumers apply
// relu(scale*y + shift) while loading (ugpg_src_t).
#include <numeric>

#include <type_traits>

#include "common.h"

namespace ugpg {

// Parallel-variance combination of one channel's per-tile partials (count, sum, M2) in ONE
// pass, shifted by K = the first non-empty tile's mean (close to the global mean, so no
// cancellation): with e_t = sum_t - n_t K,  m = K + sum e_t / N  and
// M2 = sum M2_t + sum e_t^2 / n_t - (sum e_t)^2 / N.  Whole block per channel; the result
// (N, mean, M2) is valid in thread 0.
__device__ __forceinline__ void bn_merge_tiles(const float* __restrict__ stats, int ntiles, int C,
                                               int c, double& N_o, double& mean_o, double& M2_o) {
    __shared__ double sn[16], se[16], sq[16];
    const float* cnt = stats + (size_t)c * ntiles;
    const float* sum = stats + ((size_t)C + c) * ntiles;
    const float* m2 = stats + ((size_t)2 * C + c) * ntiles;
    // this thread's first 8 tiles' partials are loaded together with the shift tile
    // (latency: the kernel is a few load round trips long)
    constexpr int PF = 8;
    float pc[PF], ps[PF], pm[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        const int t = threadIdx.x + u * blockDim.x;
        const bool ok = t < ntiles;
        pc[u] = ok ? cnt[t] : 0.f;
        ps[u] = ok ? sum[t] : 0.f;
        pm[u] = ok ? m2[t] : 0.f;
    }
    int t0 = 0;
    while (t0 < ntiles && !(cnt[t0] > 0.f)) ++t0;  // uniform: the first tile is normally full
    const double K = t0 < ntiles ? (double)sum[t0] / (double)cnt[t0] : 0.0;
    double n = 0, E = 0, M = 0;
    auto one = [&](float nb, float sm, float mm) {
        if (nb <= 0.f) return;
        const double e = (double)sm - (double)nb * K;
        n += nb;
        E += e;
        M += (double)mm + e * e * (double)(1.0f / nb);
    };
#pragma unroll
    for (int u = 0; u < PF; ++u) one(pc[u], ps[u], pm[u]);
    for (int t = threadIdx.x + PF * blockDim.x; t < ntiles; t += blockDim.x) one(cnt[t], sum[t], m2[t]);
    // fixed-order reduction: wave shuffles, then the 16 wave sums in order by thread 0
    n = wave_sum_d(n);
    E = wave_sum_d(E);
    M = wave_sum_d(M);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sn[wv] = n;
        se[wv] = E;
        sq[wv] = M;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            sn[0] += sn[w];
            se[0] += se[w];
            sq[0] += sq[w];
        }
        const double Ntot = sn[0];
        N_o = Ntot;
        mean_o = Ntot > 0 ? K + se[0] / Ntot : 0.0;
        M2_o = Ntot > 0 ? sq[0] - se[0] * se[0] / Ntot : sq[0];
    }
}

// mean/invstd/scale/shift and the running statistics (unbiased variance) of one channel
// from its merged (N, mean, M2)
__device__ __forceinline__ void bn_finalize_channel(int c, double N, double m, double M2,
                                                    const float* gamma, const float* beta,
                                                    float* rmean, float* rvar, int64_t* nbt,
                                                    float momentum, float eps, float* mean_o,
                                                    float* invstd_o, float* scale_o, float* shift_o) {
    const double var = M2 / N;
    const float inv = (float)(1.0 / sqrt(var + (double)eps));
    const float mf = (float)m;
    const float sc = inv * gamma[c];
    mean_o[c] = mf;
    invstd_o[c] = inv;
    scale_o[c] = sc;
    shift_o[c] = beta[c] - mf * sc;
    if (rmean) {
        const double unbiased = N > 1 ? M2 / (N - 1) : M2;
        rmean[c] = (float)(momentum * m + (1.0 - momentum) * (double)rmean[c]);
        rvar[c] = (float)(momentum * unbiased + (1.0 - momentum) * (double)rvar[c]);
    }
    if (c == 0 && nbt) *nbt += 1;
}

__global__ void bn_finalize_kernel(const float* __restrict__ stats, int ntiles, int C,
                                   const float* gamma, const float* beta, float* rmean,
                                   float* rvar, int64_t* nbt, float momentum, float eps,
                                   float* mean_o, float* invstd_o, float* scale_o,
                                   float* shift_o) {
    const int c = blockIdx.x;
    double N, m, M2;
    bn_merge_tiles(stats, ntiles, C, c, N, m, M2);
    if (threadIdx.x == 0)
        bn_finalize_channel(c, N, m, M2, gamma, beta, rmean, rvar, nbt, momentum, eps, mean_o,
                            invstd_o, scale_o, shift_o);
}

// ---- synchronised BatchNorm across data-parallel ranks (SURVEY §8e's optional policy) ----
// Forward: each rank merges its tiles into (N, mean, M2) in fp64 and writes them into its own
// row of a zeroed [nranks][3][C] buffer; a SUM all-reduce of that buffer is an exact gather
// (every other row is zero); every rank then merges the rows in rank order (Chan) -- the
// same bits on every rank -- and finalizes from the global statistics.
__global__ void bn_stats_pack_kernel(const float* __restrict__ stats, int ntiles, int C,
                                     double* out) {
    const int c = blockIdx.x;
    double N, m, M2;
    bn_merge_tiles(stats, ntiles, C, c, N, m, M2);
    if (threadIdx.x == 0) {
        out[c] = N;
        out[C + c] = m;
        out[2 * C + c] = M2;
    }
}

__global__ void bn_finalize_merged_kernel(const double* __restrict__ g, int nranks, int C,
                                          const float* gamma, const float* beta, float* rmean,
                                          float* rvar, int64_t* nbt, float momentum, float eps,
                                          float* mean_o, float* invstd_o, float* scale_o,
                                          float* shift_o) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double N = 0, m = 0, M2 = 0;
    for (int r = 0; r < nranks; ++r) {
        const double* row = g + (size_t)r * 3 * C;
        const double nr = row[c], mr = row[C + c], qr = row[2 * C + c];
        if (!(nr > 0)) continue;
        const double Nt = N + nr, d = mr - m;
        m += d * (nr / Nt);
        M2 += qr + d * d * (N * nr / Nt);
        N = Nt;
    }
    bn_finalize_channel(c, N, m, M2, gamma, beta, rmean, rvar, nbt, momentum, eps, mean_o, invstd_o,
                        scale_o, shift_o);
}

__global__ void bn_eval_params_kernel(const float* gamma, const float* beta, const float* rm,
                                      const float* rv, float eps, int C, float* scale,
                                      float* shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float inv = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
    const float sc = inv * gamma[c];
    scale[c] = sc;
    shift[c] = beta[c] - rm[c] * sc;
}

// Per-block partial sums of g and g*xhat over a contiguous pixel range.
// Thread layout: C/4 threads per pixel (float4 channels), 256/(C/4) pixel slots.
__global__ void __launch_bounds__(256)
    bn_bwd_reduce_kernel(const float* __restrict__ da, YRef y, int64_t npix,
                         int C, const float* mean, const float* invstd, const float* scale,
                         const float* shift, int64_t ppb, float* part, int nblk) {
    const int c4n = C / 4, slots = 256 / c4n;
    const int tid = threadIdx.x, q = tid % c4n, slot = tid / c4n;
    const int c = q * 4;
    __shared__ f32x4 rs[256], rq[256], rx[256];
    f32x4 sg = {0, 0, 0, 0}, sgx = {0, 0, 0, 0}, sx = {0, 0, 0, 0};
    if (slot < slots) {
        const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + c);
        const f32x4 is = *reinterpret_cast<const f32x4*>(invstd + c);
        const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c);
        const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c);
        const int64_t p0 = blockIdx.x * ppb, p1 = min(npix, p0 + ppb);
        auto accum = [&](f32x4 d, f32x4 v) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float g = fmaf(v[k], sc[k], sh[k]) > 0.f ? d[k] : 0.f;
                const float xh = (v[k] - mu[k]) * is[k];
                sg[k] += g;
                sgx[k] = fmaf(g, xh, sgx[k]);
                sx[k] += xh;
            }
        };
        // four pixels' loads in flight per thread before any is consumed (the loop
        // was latency-bound at one pair of 16-byte loads per thread: 4.7 TB/s)
        int64_t p = p0 + slot;
        for (; p + 3 * slots < p1; p += 4 * slots) {
            f32x4 d[4], v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                d[u] = *reinterpret_cast<const f32x4*>(da + (p + u * slots) * C + c);
                v[u] = y.ld4((p + u * slots) * C + c);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) accum(d[u], v[u]);
        }
        for (; p < p1; p += slots)
            accum(*reinterpret_cast<const f32x4*>(da + p * C + c), y.ld4(p * C + c));
    }
    rs[tid] = sg;
    rq[tid] = sgx;
    rx[tid] = sx;
    __syncthreads();
    if (slot == 0) {
        for (int s = 1; s < slots; ++s) {
            sg += rs[s * c4n + q];
            sgx += rq[s * c4n + q];
            sx += rx[s * c4n + q];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            part[(size_t)(c + k) * nblk + blockIdx.x] = sg[k];
            part[((size_t)C + c + k) * nblk + blockIdx.x] = sgx[k];
            part[((size_t)2 * C + c + k) * nblk + blockIdx.x] = sx[k];
        }
    }
}

// one channel's backward partials (sum g, sum g*xhat, sum xhat) over its slots in fp64,
// fixed order; valid in thread 0
__device__ __forceinline__ void bn_bwd_sum_slots(const float* part, int nblk, int C, int c,
                                                 double& a_o, double& b_o, double& x_o) {
    __shared__ double s1[4], s2[4], s3[4];
    double a = 0, b = 0, x = 0;
    int i = threadIdx.x;
    // four slots' loads in flight per thread (the kernel is a few load round trips long)
    for (; i + 3 * (int)blockDim.x < nblk; i += 4 * blockDim.x) {
        float va[4], vb[4], vx[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = i + u * blockDim.x;
            va[u] = part[(size_t)c * nblk + j];
            vb[u] = part[((size_t)C + c) * nblk + j];
            vx[u] = part[((size_t)2 * C + c) * nblk + j];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a += va[u];
            b += vb[u];
            x += vx[u];
        }
    }
    for (; i < nblk; i += blockDim.x) {
        a += part[(size_t)c * nblk + i];
        b += part[((size_t)C + c) * nblk + i];
        x += part[((size_t)2 * C + c) * nblk + i];
    }
    a = wave_sum_d(a);
    b = wave_sum_d(b);
    x = wave_sum_d(x);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s1[wv] = a;
        s2[wv] = b;
        s3[wv] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            s1[0] += s1[w];
            s2[0] += s2[w];
            s3[0] += s3[w];
        }
        a_o = s1[0];
        b_o = s2[0];
        x_o = s3[0];
    }
}

__global__ void bn_bwd_finalize_kernel(const float* part, int nblk, int C, int64_t npix,
                                       const float* scale, float* dgamma, float* dbeta,
                                       float* dbias, int acc, float* coef) {
    const int c = blockIdx.x;
    double A, Bs, X;
    bn_bwd_sum_slots(part, nblk, C, c, A, Bs, X);
    if (threadIdx.x == 0) {
        const float sg = (float)A, sgx = (float)Bs;
        if (dgamma) dgamma[c] = acc ? dgamma[c] + sgx : sgx;
        if (dbeta) dbeta[c] = acc ? dbeta[c] + sg : sg;
        const double mg = A / (double)npix, mgx = Bs / (double)npix;
        coef[c] = (float)mg;         // mean(g)
        coef[C + c] = (float)mgx;    // mean(g*xhat)
        if (dbias) {
            // sum_p dy_p = scale*(sum g - N*mean(g) - mean(g*xhat)*sum xhat)
            const float db = (float)((double)scale[c] * (A - (double)npix * mg - mgx * X));
            dbias[c] = acc ? dbias[c] + db : db;
        }
    }
}

// Backward of the synchronised BatchNorm: each rank's (sum g, sum g*xhat, sum xhat) in fp64
// are SUM all-reduced, then written back as ONE slot holding sum/nranks (the other slots
// zeroed), so the unchanged finalize computes mean(g) = sum_all / (nranks * npix_local) --
// the global means, as torch's SyncBatchNorm backward -- while dgamma, dbeta and the conv
// bias gradient become the global sums / nranks, whose average over ranks (the gradient
// all-reduce) is the global-batch gradient of the local-loss average.
__global__ void bn_bwd_pack_kernel(const float* part, int nblk, int C, int64_t npix, double* out) {
    const int c = blockIdx.x;
    double A, Bs, X;
    bn_bwd_sum_slots(part, nblk, C, c, A, Bs, X);
    if (threadIdx.x == 0) {
        out[c] = A;
        out[C + c] = Bs;
        out[2 * C + c] = X;
        if (c == 0) out[3 * C] = (double)npix;  // summed over ranks: the global pixel count
    }
}

// slot 0 = sum_all * npix_local / N_global: the finalize divides by npix_local, so its means
// are the global ones whatever the ranks' shard sizes (a 1/nranks scale assumed
// equal counts)
__global__ void bn_bwd_unpack_kernel(const double* __restrict__ sums, int64_t npix, float* part,
                                     int nblk, int C) {
    const double scale = (double)npix / sums[3 * C];
    const int64_t n = (int64_t)3 * C * nblk;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = i / nblk, slot = i - row * nblk;
        part[i] = slot == 0 ? (float)(sums[row] * scale) : 0.f;
    }
}

// dy = scale * (g - mean(g) - xhat * mean(g*xhat)), g = [scale*y + shift > 0] * da.
// The grid stride is a multiple of C/4 (2048 x 256 threads, C <= 1024), so each thread
// keeps one 4-channel group: its per-channel coefficients are loaded once, and four
// float4 pairs are in flight per thread.
// TY: the storage of y (float, or __bf16 under the bf16 arithmetic)
// TO: the storage of dy (float, or __bf16 = RNE of the same fp32 value: under the bf16
// arithmetic exactly what the data and weight gradients read)
// ROUTE (ugpg_bn_relu_bwd_partials_routed): da is recomputed here from what its last
// producer read instead of read back from HBM, then the base gradient (da != NULL) added --
// the same values summed in the same order as that producer, so the result is
// bit-identical to the producer writing da and this kernel reading it.
//   ROUTE_POOL: dout[pooled pixel] where the window's argmax selects this pixel (else 0)
//   ROUTE_HEAD: sum_k dh[p][k] * w[k][c], products and sums rounded separately, k in order
constexpr int ROUTE_NONE = 0, ROUTE_POOL = 1, ROUTE_HEAD = 2;
// g + d*w with the product rounded (head_bwd_kernel's arithmetic; ops.hip is built without
// contraction, this file with it)
__device__ __forceinline__ float add_prod_rn(float g, float d, float w) {
#pragma clang fp contract(off)
    return g + d * w;
}
struct Route {
    const float* src;   // POOL: NHWC [B][H/2][W/2][C]; HEAD: dh [npix][nc]
    const uint8_t* am;  // POOL: the window argmax (maxpool2_fwd)
    const float* w;     // HEAD: [nc][C]
    int nc, H, W;
};
// TD: the storage of da (float, or __bf16: the bf16 arithmetic's data gradient, ROUTE_NONE)
template <bool NT, typename TY, typename TO, int ROUTE = ROUTE_NONE, typename TD = float>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const TD* da, const TY* __restrict__ y,
                                                           int64_t npix, int C, const float* mean,
                                                           const float* invstd, const float* scale,
                                                           const float* shift, const float* coef,
                                                           TO* dy, Route rt = {}) {
    const int64_t n4 = npix * C / 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i0 >= n4) return;
    auto ld4 = [](const float* p, int c) { return *reinterpret_cast<const f32x4*>(p + c); };
    const int c = (int)((i0 * 4) % C);  // fixed: stride * 4 is a multiple of C
    // ROUTE: this thread's pixel pi, advanced by pstride pixels per grid stride; POOL also
    // keeps its (x, row, image) position, stepped without divisions
    const uint32_t pix0 = (uint32_t)((i0 * 4) / C), pstride = (uint32_t)(stride * 4 / C);
    const uint32_t W = (uint32_t)rt.W, H = (uint32_t)rt.H, Ho = H / 2, Wo = W / 2;
    uint32_t px = 0, py = 0, pb = 0, xs = 0, ys = 0, bs = 0;
    if constexpr (ROUTE == ROUTE_POOL) {
        px = pix0 % W;
        py = (pix0 / W) % H;
        pb = pix0 / W / H;
        xs = pstride % W;
        ys = (pstride / W) % H;
        bs = pstride / W / H;
    }
    auto advance = [&]() {
        if constexpr (ROUTE == ROUTE_POOL) {
            px += xs;
            const uint32_t carry = px >= W ? 1u : 0u;
            px -= carry * W;
            py += ys + carry;
            const uint32_t cy = py >= H ? 1u : 0u;
            py -= cy * H;
            pb += bs + cy;
        }
    };
    f32x4 wv[4];
    if constexpr (ROUTE == ROUTE_HEAD)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < rt.nc) wv[k] = ld4(rt.w + (size_t)k * C, c);
    auto routed = [&](uint32_t p) {
        f32x4 g = {0.f, 0.f, 0.f, 0.f};
        if constexpr (ROUTE == ROUTE_HEAD) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k >= rt.nc) break;
                const float d = rt.src[(size_t)p * rt.nc + k];
#pragma unroll
                for (int j = 0; j < 4; ++j) g[j] = add_prod_rn(g[j], d, wv[k][j]);
            }
            return g;
        }
        const uint32_t oy = py >> 1, ox = px >> 1;
        if (oy < Ho && ox < Wo) {
            const int k = (int)((py & 1) * 2 + (px & 1));
            const size_t o = ((size_t)(pb * Ho + oy) * Wo + ox) * C + c;
            const f32x4 d = *reinterpret_cast<const f32x4*>(rt.src + o);
            const uchar4 m = *reinterpret_cast<const uchar4*>(rt.am + o);
            g[0] = m.x == k ? d[0] : 0.f;
            g[1] = m.y == k ? d[1] : 0.f;
            g[2] = m.z == k ? d[2] : 0.f;
            g[3] = m.w == k ? d[3] : 0.f;
        }
        return g;
    };
    const f32x4 sc = ld4(scale, c), sh = ld4(shift, c), mu = ld4(mean, c), is = ld4(invstd, c),
                k0 = ld4(coef, c), k1 = ld4(coef, C + c);
    auto one = [&](f32x4 d, f32x4 v) {
        f32x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = bn_bwd_dy(d[k], v[k], sc[k], sh[k], mu[k], is[k], k0[k], k1[k]);
        return o;
    };
    static_assert(std::is_same<TD, float>::value || ROUTE == ROUTE_NONE, "bf16 da: no route");
    const f32x4* D = reinterpret_cast<const f32x4*>(da);
    const uint2* D16 = reinterpret_cast<const uint2*>(da);
    auto store = [&](int64_t k, f32x4 o) {
        if constexpr (std::is_same<TO, float>::value) {
            reinterpret_cast<f32x4*>(dy)[k] = o;
        } else {
            typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
            typedef float f32x2_t __attribute__((ext_vector_type(2)));
            const unsigned lo = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{o.x, o.y}, bf16x2_t));
            const unsigned hi = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{o.z, o.w}, bf16x2_t));
            reinterpret_cast<uint2*>(dy)[k] = uint2{lo, hi};
        }
    };
    auto Y = [&](int64_t k) {  // 4 values of y (a 16- or 8-byte vector)
        if constexpr (std::is_same<TY, float>::value) {
            const f32x4* q = reinterpret_cast<const f32x4*>(y) + k;
            return NT ? __builtin_nontemporal_load(q) : *q;
        } else {
            const uint2* q = reinterpret_cast<const uint2*>(y) + k;
            const uint2 u = NT ? uint2{__builtin_nontemporal_load(&q->x),
                                       __builtin_nontemporal_load(&q->y)}
                               : *q;
            return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                         __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
        }
    };
    auto DA = [&](int64_t k, uint32_t p) {  // da (read once: streaming load)
        if constexpr (ROUTE != ROUTE_NONE) {
            f32x4 g = routed(p);
            if (da) g += NT ? __builtin_nontemporal_load(D + k) : D[k];
            return g;
        } else if constexpr (std::is_same<TD, float>::value) {
            return NT ? __builtin_nontemporal_load(D + k) : D[k];
        } else {  // 4 bf16 (exact widening)
            const uint2 u = NT ? uint2{__builtin_nontemporal_load(&D16[k].x),
                                       __builtin_nontemporal_load(&D16[k].y)}
                               : D16[k];
            return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                         __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
        }
    };
    int64_t i = i0;
    uint32_t pi = pix0;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        f32x4 d[4], v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            d[u] = DA(i + u * stride, pi);
            v[u] = Y(i + u * stride);
            pi += pstride;
            advance();
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) store(i + u * stride, one(d[u], v[u]));
    }
    for (; i < n4; i += stride) {
        store(i, one(DA(i, pi), Y(i)));
        pi += pstride;
        advance();
    }
}

__global__ void bn_relu_apply_kernel(YRef x, const float* sc, const float* sh,
                                     int64_t n4, int C, float* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)((i * 4) % C);
        reinterpret_cast<f32x4*>(out)[i] = act_apply4(x.ld4((size_t)i * 4), sc, sh, c);
    }
}

// backward finalize: one thread per 8 partial slots, 64..256 (as the forward finalize)
static int bwd_fin_threads(int64_t nslots) {
    int nt = 64;
    while (nt < 256 && (int64_t)nt * 8 < nslots) nt *= 2;
    return nt;
}
constexpr int64_t kApplyBlocks = 2048;  // grid cap of the BatchNorm-backward apply
static unsigned apply_grid(int64_t n4) {
    int64_t g = cdiv(n4, 256);
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, kApplyBlocks));
}
// the apply reads da and y with streaming (nontemporal) loads -- their last use -- so dy,
// read next by the data and weight gradients, stays in the caches (step -0.55 %)
template <int ROUTE>
void launch_bn_apply_t(unsigned ga, hipStream_t st, const float* da, YRef y, int64_t npix,
                       int C, const float* mean, const float* invstd, const float* scale,
                       const float* shift, const float* coef, float* dy, __bf16* dy16,
                       Route rt, const __bf16* da16 = nullptr) {
    if constexpr (ROUTE == ROUTE_NONE) {
        if (da16) {  // (the host admits bf16 da with bf16 y and bf16 dy only)
            hipLaunchKernelGGL((bn_bwd_apply_kernel<true, __bf16, __bf16, ROUTE_NONE, __bf16>),
                               dim3(ga), dim3(256), 0, st, da16, y.h, npix, C, mean, invstd,
                               scale, shift, coef, dy16, rt);
            return;
        }
    }
    if (y.f && dy)
        hipLaunchKernelGGL((bn_bwd_apply_kernel<true, float, float, ROUTE>), dim3(ga), dim3(256),
                           0, st, da, y.f, npix, C, mean, invstd, scale, shift, coef, dy, rt);
    else if (y.f)
        hipLaunchKernelGGL((bn_bwd_apply_kernel<true, float, __bf16, ROUTE>), dim3(ga), dim3(256),
                           0, st, da, y.f, npix, C, mean, invstd, scale, shift, coef, dy16, rt);
    else if (dy)
        hipLaunchKernelGGL((bn_bwd_apply_kernel<true, __bf16, float, ROUTE>), dim3(ga), dim3(256),
                           0, st, da, y.h, npix, C, mean, invstd, scale, shift, coef, dy, rt);
    else
        hipLaunchKernelGGL((bn_bwd_apply_kernel<true, __bf16, __bf16, ROUTE>), dim3(ga),
                           dim3(256), 0, st, da, y.h, npix, C, mean, invstd, scale, shift, coef,
                           dy16, rt);
}
void launch_bn_apply(unsigned ga, hipStream_t st, const float* da, YRef y, int64_t npix,
                     int C, const float* mean, const float* invstd, const float* scale,
                     const float* shift, const float* coef, float* dy, __bf16* dy16,
                     int kind = ROUTE_NONE, Route rt = {}, const __bf16* da16 = nullptr) {
    if (kind == ROUTE_POOL)
        launch_bn_apply_t<ROUTE_POOL>(ga, st, da, y, npix, C, mean, invstd, scale, shift, coef,
                                      dy, dy16, rt);
    else if (kind == ROUTE_HEAD)
        launch_bn_apply_t<ROUTE_HEAD>(ga, st, da, y, npix, C, mean, invstd, scale, shift, coef,
                                      dy, dy16, rt);
    else
        launch_bn_apply_t<ROUTE_NONE>(ga, st, da, y, npix, C, mean, invstd, scale, shift, coef,
                                      dy, dy16, rt, da16);
}
constexpr int64_t kBwdBlocks = 2048, kBwdPpt = 8;
namespace {
struct BwdPlan {
    int nblk;
    int64_t ppb;
};
// Reduce blocks: as many as keep >= ppt pixels per thread (a block covers 256 / (C/4)
// pixels per pass), at most kBwdBlocks: the narrow-pixel, wide-channel layers
// (C = 512 at 32^2 / 16^2) need many blocks for enough loads in flight -- the former
// npix/64 rule gave them 1 block per CU (latency-bound, SQ_WAIT_ANY 0.93).
BwdPlan bwd_plan(int64_t npix, int C) {
    BwdPlan p;
    const int slots = 256 / (C / 4 > 0 ? C / 4 : 1);
    int64_t nb = npix / ((int64_t)slots * kBwdPpt);
    if (nb > kBwdBlocks) nb = kBwdBlocks;
    if (nb < 1) nb = 1;
    p.ppb = cdiv(npix, nb);
    p.nblk = (int)cdiv(npix, p.ppb);
    return p;
}
}  // namespace
}  // namespace ugpg

using namespace ugpg;

// threads per channel of the forward merge: one per PF = 8 slots, 64..1024
static int fwd_fin_threads(int ntiles) {
    int nt = 64;
    while (nt < 1024 && (int64_t)nt * 8 < ntiles) nt *= 2;
    return nt;
}

extern "C" int ugpg_bn_finalize(const float* stats, int ntiles, int C, const float* gamma,
                                const float* beta, float* running_mean, float* running_var,
                                int64_t* nbt, float momentum, float eps, float* mean,
                                float* invstd, float* scale, float* shift, void* stream) {
    if (!stats || !gamma || !beta || !mean || !invstd || !scale || !shift || C <= 0 ||
        ntiles <= 0 || (!running_mean != !running_var)) {
        set_error("bn_finalize: bad arguments");
        return UGPG_ERR_INVALID;
    }
    // threads per channel: one per PF = 8 slots, 64..1024 -- the narrow-image layers have
    // 128-512 slots, and 1024-thread blocks of mostly idle lanes cost them ~4 us a launch
    const int nt = fwd_fin_threads(ntiles);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(nt), 0, as_stream(stream), stats,
                       ntiles, C, gamma, beta, running_mean, running_var, nbt, momentum, eps,
                       mean, invstd, scale, shift);
    return check_launch("bn_finalize");
}

extern "C" int ugpg_bn_stats_pack(const float* stats, int ntiles, int C, double* out,
                                  void* stream) {
    if (!stats || !out || C <= 0 || ntiles <= 0) {
        set_error("bn_stats_pack: bad arguments");
        return UGPG_ERR_INVALID;
    }
    hipLaunchKernelGGL(bn_stats_pack_kernel, dim3(C), dim3(fwd_fin_threads(ntiles)), 0,
                       as_stream(stream), stats, ntiles, C, out);
    return check_launch("bn_stats_pack");
}

extern "C" int ugpg_bn_finalize_merged(const double* merged, int nranks, int C, const float* gamma,
                                       const float* beta, float* running_mean, float* running_var,
                                       int64_t* nbt, float momentum, float eps, float* mean,
                                       float* invstd, float* scale, float* shift, void* stream) {
    if (!merged || nranks <= 0 || !gamma || !beta || !mean || !invstd || !scale || !shift ||
        C <= 0 || (!running_mean != !running_var)) {
        set_error("bn_finalize_merged: bad arguments");
        return UGPG_ERR_INVALID;
    }
    hipLaunchKernelGGL(bn_finalize_merged_kernel, dim3(cdiv(C, 256)), dim3(256), 0,
                       as_stream(stream), merged, nranks, C, gamma, beta, running_mean, running_var,
                       nbt, momentum, eps, mean, invstd, scale, shift);
    return check_launch("bn_finalize_merged");
}

extern "C" int ugpg_bn_eval_params(const float* gamma, const float* beta, const float* rm,
                                   const float* rv, float eps, int C, float* scale, float* shift,
                                   void* stream) {
    if (!gamma || !beta || !rm || !rv || !scale || !shift || C <= 0) {
        set_error("bn_eval_params: bad arguments");
        return UGPG_ERR_INVALID;
    }
    hipLaunchKernelGGL(bn_eval_params_kernel, dim3(cdiv(C, 256)), dim3(256), 0,
                       as_stream(stream), gamma, beta, rm, rv, eps, C, scale, shift);
    return check_launch("bn_eval_params");
}

extern "C" size_t ugpg_bn_relu_bwd_workspace(int64_t npix, int C) {
    BwdPlan p = bwd_plan(npix, C);
    return ((size_t)3 * C * p.nblk + (size_t)2 * C) * sizeof(float);
}

extern "C" int ugpg_bn_relu_bwd(const float* da, const float* y_f32, const void* y_bf16,
                                int64_t npix, int C, const float* mean, const float* invstd,
                                const float* scale, const float* shift, float* dy, void* dy_bf16,
                                float* dgamma, float* dbeta, float* dbias, int acc, void* ws,
                                size_t ws_bytes, void* stream) {
    const YRef y = yref(y_f32, y_bf16);
    if (!da || (!y.f && !y.h) || !dy == !dy_bf16 || !mean || !invstd || !scale || !shift ||
        C % 4 || C > 1024 || npix <= 0) {
        set_error("bn_relu_bwd: bad arguments (C=%d)", C);
        return UGPG_ERR_INVALID;
    }
    const size_t need = ugpg_bn_relu_bwd_workspace(npix, C);
    if (!ws || ws_bytes < need) {
        set_error("bn_relu_bwd: workspace %zu < %zu", ws_bytes, need);
        return UGPG_ERR_WORKSPACE;
    }
    BwdPlan p = bwd_plan(npix, C);
    float* part = static_cast<float*>(ws);
    float* coef = part + (size_t)3 * C * p.nblk;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(p.nblk), dim3(256), 0, st, da, y, npix, C, mean,
                       invstd, scale, shift, p.ppb, part, p.nblk);
    if (int e = check_launch("bn_bwd_reduce")) return e;
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(bwd_fin_threads(p.nblk)), 0, st, part,
                       p.nblk, C, npix, scale, dgamma, dbeta, dbias, acc, coef);
    if (int e = check_launch("bn_bwd_finalize")) return e;
    // the apply kernel keeps one channel group per thread: grid * 1024 must be a multiple of C
    const unsigned q = (unsigned)(C / std::gcd(1024, C));
    const unsigned ga = (apply_grid(npix * C / 4) + q - 1) / q * q;
    launch_bn_apply(ga, st, da, y, npix, C, mean, invstd, scale, shift, coef, dy,
                    static_cast<__bf16*>(dy_bf16));
    return check_launch("bn_bwd_apply");
}

namespace ugpg {
void launch_bn_bwd_reduce(const float* da, YRef y, int64_t npix, int C, const float* mean,
                          const float* invstd, const float* scale, const float* shift, float* part,
                          int nslots, hipStream_t st) {
    const int64_t ppb = cdiv(npix, (int64_t)nslots);
    // blocks past the pixels (nslots > npix) write zero partials
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nslots), dim3(256), 0, st, da, y, npix, C, mean,
                       invstd, scale, shift, ppb, part, nslots);
}
}  // namespace ugpg

extern "C" int ugpg_bnb_slots(int64_t npix, int C) {
    if (npix <= 0 || C <= 0 || C % 4 || C > 1024) return 0;
    return bwd_plan(npix, C).nblk;
}

extern "C" int ugpg_bn_relu_bwd_reduce(const float* da, const float* y_f32, const void* y_bf16,
                                       int64_t npix, int C, const float* mean, const float* invstd,
                                       const float* scale, const float* shift, float* part,
                                       int nslots, void* stream) {
    const YRef y = yref(y_f32, y_bf16);
    if (!da || (!y.f && !y.h) || !mean || !invstd || !scale || !shift || !part || nslots <= 0 ||
        C % 4 || C <= 0 || C > 1024 || npix <= 0) {
        set_error("bn_relu_bwd_reduce: bad arguments (C=%d nslots=%d)", C, nslots);
        return UGPG_ERR_INVALID;
    }
    launch_bn_bwd_reduce(da, y, npix, C, mean, invstd, scale, shift, part, nslots,
                         as_stream(stream));
    return check_launch("bn_bwd_reduce");
}

extern "C" int ugpg_bn_bwd_partials_pack(const float* part, int nslots, int C, int64_t npix,
                                         double* out, void* stream) {
    if (!part || !out || nslots <= 0 || C <= 0 || npix <= 0) {
        set_error("bn_bwd_partials_pack: bad arguments");
        return UGPG_ERR_INVALID;
    }
    hipLaunchKernelGGL(bn_bwd_pack_kernel, dim3(C), dim3(bwd_fin_threads(nslots)), 0,
                       as_stream(stream), part, nslots, C, npix, out);
    return check_launch("bn_bwd_partials_pack");
}

extern "C" int ugpg_bn_bwd_partials_unpack(const double* sums, int64_t npix, float* part,
                                           int nslots, int C, void* stream) {
    if (!sums || !part || nslots <= 0 || C <= 0 || npix <= 0) {
        set_error("bn_bwd_partials_unpack: bad arguments");
        return UGPG_ERR_INVALID;
    }
    const int64_t n = (int64_t)3 * C * nslots;
    hipLaunchKernelGGL(bn_bwd_unpack_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 1024)),
                       dim3(256), 0, as_stream(stream), sums, npix, part, nslots, C);
    return check_launch("bn_bwd_partials_unpack");
}

extern "C" size_t ugpg_bn_relu_bwd_partials_workspace(int C) {
    return C > 0 ? (size_t)2 * C * sizeof(float) : 0;
}

// finalize + apply of ugpg_bn_relu_bwd from partials a data gradient wrote (bnb_part);
// rt: da routed from a max-pool's output gradient (da = NULL: no base gradient)
static int bn_relu_bwd_partials(int kind, const Route& rt, const float* part, int nslots,
                                const float* da, const float* y_f32, const void* y_bf16,
                                int64_t npix, int C, const float* mean, const float* invstd,
                                const float* scale, const float* shift, float* dy, void* dy_bf16,
                                float* dgamma, float* dbeta, float* dbias, int acc, void* ws,
                                size_t ws_bytes, void* stream, const void* da_bf16 = nullptr) {
    const YRef y = yref(y_f32, y_bf16);
    // dy == dy_bf16 == NULL: the finalize only (the apply's coefficients stay in ws for a
    // weight gradient that forms dy while loading, ugpg_wgrad_t.dy_bn)
    const bool fin_only = !dy && !dy_bf16 && kind == ROUTE_NONE;
    if (!part || nslots <= 0 || (!da && !da_bf16 && kind == ROUTE_NONE && !fin_only) ||
        (da && da_bf16) || (!y.f && !y.h) || (dy && dy_bf16) || (!dy && !dy_bf16 && !fin_only) ||
        !mean || !invstd || !scale || !shift || C % 4 || C <= 0 || C > 1024 || npix <= 0) {
        set_error("bn_relu_bwd_partials: bad arguments (C=%d nslots=%d)", C, nslots);
        return UGPG_ERR_INVALID;
    }
    if (da_bf16 && !fin_only && (kind != ROUTE_NONE || y.f || dy)) {
        set_error("bn_relu_bwd_partials: a bf16 da needs a bf16 y and a bf16 dy");
        return UGPG_ERR_INVALID;
    }
    const size_t need = ugpg_bn_relu_bwd_partials_workspace(C);
    if (!ws || ws_bytes < need) {
        set_error("bn_relu_bwd_partials: workspace %zu < %zu", ws_bytes, need);
        return UGPG_ERR_WORKSPACE;
    }
    float* coef = static_cast<float*>(ws);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(bwd_fin_threads(nslots)), 0, st,
                       part, nslots, C, npix, scale, dgamma, dbeta, dbias, acc, coef);
    if (int e = check_launch("bn_bwd_finalize")) return e;
    if (fin_only) return UGPG_OK;
    const unsigned q = (unsigned)(C / std::gcd(1024, C));
    const unsigned ga = (apply_grid(npix * C / 4) + q - 1) / q * q;
    launch_bn_apply(ga, st, da, y, npix, C, mean, invstd, scale, shift, coef, dy,
                    static_cast<__bf16*>(dy_bf16), kind, rt, static_cast<const __bf16*>(da_bf16));
    return check_launch("bn_bwd_apply");
}

extern "C" int ugpg_bn_relu_bwd_partials(const float* part, int nslots, const float* da,
                                         const void* da_bf16, const float* y_f32,
                                         const void* y_bf16, int64_t npix, int C,
                                         const float* mean, const float* invstd,
                                         const float* scale, const float* shift, float* dy,
                                         void* dy_bf16, float* dgamma, float* dbeta, float* dbias,
                                         int acc, void* ws, size_t ws_bytes, void* stream) {
    return bn_relu_bwd_partials(ROUTE_NONE, Route{}, part, nslots, da, y_f32, y_bf16, npix, C,
                                mean, invstd, scale, shift, dy, dy_bf16, dgamma, dbeta, dbias, acc,
                                ws, ws_bytes, stream, da_bf16);
}

extern "C" int ugpg_bn_relu_bwd_partials_routed(const ugpg_bwd_route_t* route, const float* part,
                                                int nslots, const float* da, const float* y_f32,
                                                const void* y_bf16, int64_t npix, int C,
                                                const float* mean, const float* invstd,
                                                const float* scale, const float* shift, float* dy,
                                                void* dy_bf16, float* dgamma, float* dbeta,
                                                float* dbias, int acc, void* ws, size_t ws_bytes,
                                                void* stream) {
    const bool pool = route && route->kind == UGPG_ROUTE_MAXPOOL2 && route->argmax &&
                      route->B > 0 && route->H > 0 && route->W > 0 &&
                      (int64_t)route->B * route->H * route->W == npix;
    const bool head = route && route->kind == UGPG_ROUTE_HEAD && route->w && route->nc >= 1 &&
                      route->nc <= 4;
    if (!route || !route->src || (!pool && !head) || npix > INT32_MAX) {
        set_error("bn_relu_bwd_partials_routed: bad route (npix=%lld)", (long long)npix);
        return UGPG_ERR_INVALID;
    }
    const Route rt{route->src, route->argmax, route->w, route->nc, route->H, route->W};
    return bn_relu_bwd_partials(pool ? ROUTE_POOL : ROUTE_HEAD, rt, part, nslots, da, y_f32,
                                y_bf16, npix, C, mean, invstd, scale, shift, dy, dy_bf16, dgamma,
                                dbeta, dbias, acc, ws, ws_bytes, stream);
}

extern "C" int ugpg_bn_relu_apply(ugpg_src_t src, int64_t npix, float* out, void* stream) {
    if ((!src.data && !src.data_bf16) || !out || src.C % 4) {
        set_error("bn_relu_apply: bad arguments");
        return UGPG_ERR_INVALID;
    }
    const int64_t n4 = npix * src.C / 4;
    hipLaunchKernelGGL(bn_relu_apply_kernel, dim3(stream_grid(n4)), dim3(256), 0,
                       as_stream(stream), yref(src), src.scale, src.shift, n4, src.C, out);
    return check_launch("bn_relu_apply");
}
