// warp_exp.hip — profiling harness (not part of the product): experimental forms of the refinement ROI sampling
// (K6b) timed against the product k_roi_warp on the microbenchmark's Src7 layer-0 problem, outputs compared byte for
// byte with the product's.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/warp_exp.hip -o build/warp_exp
#include "../fastest_image_pattern_matching_amd/csrc/fpm_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace fpm;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// exact bilinear taps from an LDS byte offset (address space 3: plain ds_read with no base add)
typedef __attribute__((address_space(3))) const uint8_t lds_u8;
typedef __attribute__((address_space(3))) const uint16_t lds_u16;
// four byte reads, 24-bit multiplies only
__device__ __forceinline__ int tap_b(uint32_t off, int ftw, int fx, int fy) {
    lds_u8* p = (lds_u8*)(size_t)off;
    lds_u8* q = (lds_u8*)(size_t)(off + ftw);
    const int v0 = p[0], v1 = p[1], v2 = q[0], v3 = q[1];
    const int h0 = mad24(fx, v1 - v0, v0 << 5), h1 = mad24(fx, v3 - v2, v2 << 5);
    return mad24(fy, h1 - h0, (h0 << 5) + 512) >> 10;
}
// two (possibly unaligned) u16 reads, horizontal pass by u8 dot products
__device__ __forceinline__ int tap_u16(uint32_t off, int ftw, int fx, int fy) {
    const uint32_t r0 = *(lds_u16*)(size_t)off, r1 = *(lds_u16*)(size_t)(off + ftw);
    const uint32_t wx = (uint32_t)mad24(fx, 255, 32);
    const int h0 = (int)__builtin_amdgcn_udot4(r0, wx, 0u, false), h1 = (int)__builtin_amdgcn_udot4(r1, wx, 0u, false);
    return mad24(fy, h1 - h0, (h0 << 5) + 512) >> 10;
}

// footprint staging by 16-byte loads: every row split into Q <= 5 aligned 16-byte chunks, 64 / Q rows per wave
// instruction, up to 4 instructions (48 rows at Q = 5) issued before any LDS write; the LDS image keeps the product's
// layout (row pitch ftw, row start bxa)
__device__ __forceinline__ void stage_footprint16(uint8_t* FT, int ftw, int fth, const uint8_t* lvl, size_t P, int bxa,
                                                  int by0, int lane) {
    const int x16 = bxa & ~15, sh = bxa - x16;
    const int Q = (sh + ftw + 15) >> 4;
    const int rpi = 64 / Q;                      // rows per instruction
    const int r = lane / Q, q = lane - r * Q;
    const uint8_t* g = lvl + (size_t)by0 * P + x16 + 16 * q;
    const bool colok = x16 + 16 * q < (int)P && lane < rpi * Q;
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = r + rpi * i;
        v[i] = (colok && row < fth) ? *(const uint4*)(g + (size_t)row * P) : make_uint4(0, 0, 0, 0);
    }
    const int wpr = ftw >> 2;
    const int d0 = (16 * q - sh) >> 2;           // first destination dword of this chunk (may be < 0)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = r + rpi * i;
        if (!colok || row >= fth) continue;
        uint32_t* dr = (uint32_t*)(FT + row * ftw);
        const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (d0 + k >= 0 && d0 + k < wpr) dr[d0 + k] = w[k];
    }
}

// TAP 2 (bytes) / 3 (u16 + dot4) on interior tiles: the row coordinates are offset per tile by whole multiples of 2^10
// so that (X0 + ad) >> 10 is the tap's column inside the wave's footprint plus the footprint's LDS byte offset, and
// (Y0 + bd) >> 10 its footprint row: address = mad24(row, ftw, col), fractions untouched
template <int TAP>
__global__ __launch_bounds__(256) void k_warp_t(RoiArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t ft_all[4 * ROI_FT + 16];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t* FT = ft_all + wv * ROI_FT;
    const uint32_t ft_lds = (uint32_t)(size_t)(lds_u8*)FT;
    const int RW = a.tw + 6, RH = a.th + 6, W = a.W, H = a.H;
    const int txn = (RW + ROI_T - 1) / ROI_T, tyn = (RH + ROI_T - 1) / ROI_T;
    const int per_roi = txn * tyn;
    const int tasks = roi_count(a) * per_roi;
    const int lr = lane >> 3, lg = lane & 7;
    const XcdSplit xs = xcd_split(tasks);
    const int tstride = xs.nk * 4;
    for (int task = xs.lo + xs.k * 4 + wv; task < xs.hi; task += tstride) {
        const int slot = task / per_roi;
        const int rem = task - slot * per_roi;
        const int ty = rem / txn, tx = rem - ty * txn;
        const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
        const int ry0 = ty * ROI_T, ry1 = min(ry0 + ROI_T, RH) - 1;
        const int c0 = cx0 + 4 * lg;
        WarpTask cur;
        warp_task_load(a, task, xs.hi, per_roi, txn, RW, RH, lr, lg, cur);
        const int4 dsc = cur.dsc, A = cur.A, B = cur.B;
        const uint8_t* lvl = cur.lvl;
        const int bxa = dsc.x, by0 = dsc.y, ftw = dsc.z & 0xffff, fth = dsc.z >> 16, flags = dsc.w;
        const bool in_lds = (flags & kTileLds) != 0;
        const int wpr = ftw >> 2;
        wave_sync();
        if ((flags & kTileAny) && in_lds) {
            if (TAP >= 6 && fth <= 48) stage_footprint16(FT, ftw, fth, lvl, a.P, bxa, by0, lane);
            else stage_footprint<2>(FT, ftw, wpr, fth, lvl + (size_t)by0 * a.P + bxa, a.P, bxa, a.P, lane);
        }
        wave_sync();
        if (c0 > cx1) continue;
        uint8_t* dst = a.roi + (size_t)slot * a.roi_stride + ((size_t)(ty * txn + tx) << 10) + 4 * lg - (size_t)ry0 * ROI_T;
        const int adv[4] = {A.x, A.y, A.z, A.w}, bdv[4] = {B.x, B.y, B.z, B.w};
        if ((flags & kTileInterior) && in_lds && TAP >= 4) {
            // TAP 4 / 5: every byte of RB rows (4 pixels each) read before any arithmetic (ILP over the LDS latency)
            constexpr int RB = TAP == 5 ? 2 : 1;
            const int nvalid = RW - c0;
            const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (1u << (8 * nvalid)) - 1u;
            const int xo = ((int)ft_lds - bxa) << kAbBits, yo = -(by0 << kAbBits);
#pragma unroll
            for (int i0 = 0; i0 < 4; i0 += RB) {
                uint32_t off[RB][4];
                int fxv[RB][4], fyv[RB][4];
                int v[RB][4][4];
#pragma unroll
                for (int k = 0; k < RB; ++k) {
                    const int x0r = cur.X0r[i0 + k] + xo, y0r = cur.Y0r[i0 + k] + yo;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int sxv = x0r + adv[u], syv = y0r + bdv[u];
                        fxv[k][u] = __builtin_amdgcn_ubfe(sxv, kAbBits - kInterBits, kInterBits);
                        fyv[k][u] = __builtin_amdgcn_ubfe(syv, kAbBits - kInterBits, kInterBits);
                        off[k][u] = (uint32_t)mad24(syv >> kAbBits, ftw, sxv >> kAbBits);
                    }
                }
#pragma unroll
                for (int k = 0; k < RB; ++k)
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        lds_u8* p = (lds_u8*)(size_t)off[k][u];
                        lds_u8* q = (lds_u8*)(size_t)(off[k][u] + ftw);
                        v[k][u][0] = p[0]; v[k][u][1] = p[1]; v[k][u][2] = q[0]; v[k][u][3] = q[1];
                    }
#pragma unroll
                for (int k = 0; k < RB; ++k) {
                    const int r = ry0 + lr + 8 * (i0 + k);
                    uint32_t pk = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int fx = fxv[k][u], fy = fyv[k][u];
                        const int h0 = mad24(fx, v[k][u][1] - v[k][u][0], v[k][u][0] << 5);
                        const int h1 = mad24(fx, v[k][u][3] - v[k][u][2], v[k][u][2] << 5);
                        pk |= (uint32_t)(mad24(fy, h1 - h0, (h0 << 5) + 512) >> 10) << (8 * u);
                    }
                    if (r <= ry1) *(uint32_t*)(dst + (size_t)r * ROI_T) = pk & colmask;
                }
            }
            continue;
        }
        if ((flags & kTileInterior) && in_lds) {
            const int nvalid = RW - c0;
            const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (1u << (8 * nvalid)) - 1u;
            const int xo = ((int)ft_lds - bxa) << kAbBits, yo = -(by0 << kAbBits);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = ry0 + lr + 8 * i;
                if (r > ry1) break;
                const int x0r = cur.X0r[i] + xo, y0r = cur.Y0r[i] + yo;
                uint32_t pk = 0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int sxv = x0r + adv[u], syv = y0r + bdv[u];
                    const int fx = __builtin_amdgcn_ubfe(sxv, kAbBits - kInterBits, kInterBits);
                    const int fy = __builtin_amdgcn_ubfe(syv, kAbBits - kInterBits, kInterBits);
                    const uint32_t off = (uint32_t)mad24(syv >> kAbBits, ftw, sxv >> kAbBits);
                    const int v = TAP == 3 ? tap_u16(off, ftw, fx, fy) : tap_b(off, ftw, fx, fy);
                    pk |= (uint32_t)v << (8 * u);
                }
                *(uint32_t*)(dst + (size_t)r * ROI_T) = pk & colmask;
            }
            continue;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = ry0 + lr + 8 * i;
            if (r > ry1) break;
            uint32_t pk = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int X = (cur.X0r[i] + adv[u]) >> (kAbBits - kInterBits);
                const int Y = (cur.Y0r[i] + bdv[u]) >> (kAbBits - kInterBits);
                int v = in_lds ? ft_tap_general(FT, ftw, bxa, by0, W, H, X, Y) : roi_tap(lvl, W, H, a.P, X, Y);
                if (c0 + u >= RW) v = 0;
                pk |= (uint32_t)v << (8 * u);
            }
            *(uint32_t*)(dst + (size_t)r * ROI_T) = pk;
        }
    }
}

// ---- experimental K6b: footprint of the NEXT tile loaded into registers during this tile's gathers (software
// pipeline: no staging latency in the wave's critical path), TAP 0 = byte gathers, 1 = dword-pair dot4 taps
template <int TAP, bool PIPE>
__global__ __launch_bounds__(256) void k_warp_x(RoiArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t ft_all[4 * ROI_FT + 16];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t* FT = ft_all + wv * ROI_FT;
    const int RW = a.tw + 6, RH = a.th + 6, W = a.W, H = a.H;
    const int txn = (RW + ROI_T - 1) / ROI_T, tyn = (RH + ROI_T - 1) / ROI_T;
    const int per_roi = txn * tyn;
    const int tasks = roi_count(a) * per_roi;
    const int lr = lane >> 3, lg = lane & 7;
    const XcdSplit xs = xcd_split(tasks);
    const int tstride = xs.nk * 4;
    int task = xs.lo + xs.k * 4 + wv;
    WarpTask cur, nxt;
    uint32_t fv[16];
    auto staged = [](const WarpTask& w) { return (w.dsc.w & kTileAny) && (w.dsc.w & kTileLds); };
    auto load_foot = [&](const WarpTask& w) {
        const int wpr = (w.dsc.z & 0xffff) >> 2, fth = w.dsc.z >> 16, total = wpr * fth;
        const uint8_t* g = w.lvl + (size_t)w.dsc.y * a.P + w.dsc.x;
        int r = lane / wpr, c = lane - (lane / wpr) * wpr;
        const int dr = 64 / wpr, dc = 64 - dr * wpr;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            fv[i] = (lane + 64 * i < total) ? *(const uint32_t*)(g + (size_t)r * a.P + 4 * c) : 0u;
            r += dr;
            c += dc;
            if (c >= wpr) { c -= wpr; ++r; }
        }
    };
    auto store_foot = [&](const WarpTask& w) {
        const int total = ((w.dsc.z & 0xffff) >> 2) * (w.dsc.z >> 16);
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (lane + 64 * i < total) ((uint32_t*)FT)[lane + 64 * i] = fv[i];
    };
    if (task < xs.hi) {
        warp_task_load(a, task, xs.hi, per_roi, txn, RW, RH, lr, lg, cur);
        if (staged(cur)) load_foot(cur);
    }
    for (; task < xs.hi; task += tstride) {
        wave_sync();   // previous task's gathers are done with FT
        if (staged(cur)) store_foot(cur);
        wave_sync();
        const int ntask = task + tstride;
        if (PIPE && ntask < xs.hi) {
            warp_task_load(a, ntask, xs.hi, per_roi, txn, RW, RH, lr, lg, nxt);
            if (staged(nxt)) load_foot(nxt);
        }
        const int slot = task / per_roi;
        const int rem = task - slot * per_roi;
        const int ty = rem / txn, tx = rem - ty * txn;
        const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
        const int ry0 = ty * ROI_T, ry1 = min(ry0 + ROI_T, RH) - 1;
        const int c0 = cx0 + 4 * lg;
        const int4 dsc = cur.dsc, A = cur.A, B = cur.B;
        const uint8_t* lvl = cur.lvl;
        const int bxa = dsc.x, by0 = dsc.y, ftw = dsc.z & 0xffff, flags = dsc.w;
        const bool in_lds = (flags & kTileLds) != 0;
        if (c0 <= cx1) {
            uint8_t* dst = a.roi + (size_t)slot * a.roi_stride + ((size_t)(ty * txn + tx) << 10) + 4 * lg - (size_t)ry0 * ROI_T;
            const int adv[4] = {A.x, A.y, A.z, A.w}, bdv[4] = {B.x, B.y, B.z, B.w};
            if ((flags & kTileInterior) && in_lds) {
                const int obase = by0 * ftw + bxa;
                const int nvalid = RW - c0;
                const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (1u << (8 * nvalid)) - 1u;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = ry0 + lr + 8 * i;
                    if (r > ry1) break;
                    uint32_t pk = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int X = (cur.X0r[i] + adv[u]) >> (kAbBits - kInterBits);
                        const int Y = (cur.Y0r[i] + bdv[u]) >> (kAbBits - kInterBits);
                        const int off = mad24(Y >> kInterBits, ftw, (X >> kInterBits) - obase);
                        const int v = TAP == 1 ? ft_tap_interior(FT, off, ftw, X, Y) : ft_tap_bytes(FT, off, ftw, X, Y);
                        pk |= (uint32_t)v << (8 * u);
                    }
                    *(uint32_t*)(dst + (size_t)r * ROI_T) = pk & colmask;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = ry0 + lr + 8 * i;
                    if (r > ry1) break;
                    uint32_t pk = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int X = (cur.X0r[i] + adv[u]) >> (kAbBits - kInterBits);
                        const int Y = (cur.Y0r[i] + bdv[u]) >> (kAbBits - kInterBits);
                        int v = in_lds ? ft_tap_general(FT, ftw, bxa, by0, W, H, X, Y) : roi_tap(lvl, W, H, a.P, X, Y);
                        if (c0 + u >= RW) v = 0;
                        pk |= (uint32_t)v << (8 * u);
                    }
                    *(uint32_t*)(dst + (size_t)r * ROI_T) = pk;
                }
            }
        }
        if (PIPE) {
            cur = nxt;
        } else if (ntask < xs.hi) {
            warp_task_load(a, ntask, xs.hi, per_roi, txn, RW, RH, lr, lg, cur);
            if (staged(cur)) load_foot(cur);
        }
    }
}

int main(int argc, char** argv) {
    auto envi = [](const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; };
    const int W = envi("MB_W", 4024), H = envi("MB_H", 3036), P = envi("MB_P", 4096), TW = envi("MB_TW", 762),
              TH = envi("MB_TH", 521);
    const int nsrc = envi("MB_NSRC", 8), ncand = 11, n3 = 3;
    const float sc = W / 4024.f;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    std::vector<uint8_t> img((size_t)P * (H + 1) * nsrc);
    srand(1);
    for (auto& v : img) v = rand() & 255;
    uint8_t* d_img;
    CK(hipMalloc(&d_img, img.size()));
    CK(hipMemcpy(d_img, img.data(), img.size(), hipMemcpyHostToDevice));
    const int C = nsrc * ncand;
    std::vector<CandState> st(C);
    std::vector<int> live(C);
    std::vector<AngleNode> nodes(C * n3);
    for (int i = 0; i < C; ++i) {
        st[i].lt = f2(sc * (300.f + 137.f * (i % 11)) / 2, sc * (200.f + 91.f * (i % 7)) / 2);
        st[i].node = i; st[i].alive = 1; st[i].reached0 = 1;
        live[i] = i;
        for (int j = 0; j < n3; ++j) {
            const double ang = -170.0 + 31.7 * i + 0.075 * (j - 1), r = ang * kD2R;
            nodes[i * n3 + j] = {ang, cos(r), sin(r), cos(-r), sin(-r)};
        }
    }
    CandState* d_st; int *d_live, *d_cnt; AngleNode* d_nodes;
    CK(hipMalloc(&d_st, sizeof(CandState) * C)); CK(hipMalloc(&d_live, 4 * C)); CK(hipMalloc(&d_cnt, 4));
    CK(hipMalloc(&d_nodes, sizeof(AngleNode) * C * n3));
    CK(hipMemcpy(d_st, st.data(), sizeof(CandState) * C, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_live, live.data(), 4 * C, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_cnt, &C, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_nodes, nodes.data(), sizeof(AngleNode) * C * n3, hipMemcpyHostToDevice));
    RoiArgs a{};
    a.level = d_img; a.level_stride = (size_t)P * (H + 1); a.W = W; a.H = H; a.P = P;
    a.tw = TW; a.th = TH;
    a.n3 = n3; a.per_source = ncand; a.slot_base = 0; a.slot_cap = C * n3;
    a.live = d_live; a.live_count = d_cnt; a.state = d_st; a.nodes = d_nodes;
    a.tabw = roi_pitch_for(TW); a.tabh = roi_tab_rows(TH);
    a.roi_pitch = roi_pitch_for(TW); a.roi_stride = roi_tiles_bytes(TW, TH);
    CK(hipMalloc(&a.tab, (size_t)C * n3 * 2 * (a.tabw + a.tabh) * 4));
    a.tdesc_stride = roi_tiles_for(TW, TH);
    CK(hipMalloc(&a.tdesc, (size_t)C * n3 * a.tdesc_stride * sizeof(int4)));
    const size_t roi_bytes = (size_t)C * n3 * a.roi_stride;
    CK(hipMalloc(&a.roi, roi_bytes));
    uint8_t* ref_roi;
    CK(hipMalloc(&ref_roi, roi_bytes));
    auto timeit = [&](auto fn, const char* name) {
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        fn();
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %8.1f us\n", name, ms * 1000.f / reps);
    };
    launch_roi_tables(a, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemset(a.roi, 0, roi_bytes));
    timeit([&] { launch_roi_warp(a, 0); }, "product warp");
    CK(hipMemcpy(ref_roi, a.roi, roi_bytes, hipMemcpyDeviceToDevice));
    std::vector<uint8_t> h_ref(roi_bytes), h_got(roi_bytes);
    CK(hipMemcpy(h_ref.data(), ref_roi, roi_bytes, hipMemcpyDeviceToHost));
    const long tiles = (long)a.slot_cap * ((TH + 6 + 31) / 32) * ((TW + 6 + 31) / 32);
    const int grid = (int)std::min<long>((tiles + 3) / 4, 16384);
    auto check = [&](const char* name) {
        CK(hipMemcpy(h_got.data(), a.roi, roi_bytes, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < roi_bytes; ++i) bad += h_got[i] != h_ref[i];
        printf("  %-26s %s (%zu bytes differ)\n", name, bad ? "MISMATCH" : "identical", bad);
        CK(hipMemset(a.roi, 0, roi_bytes));
    };
    CK(hipMemset(a.roi, 0, roi_bytes));
    timeit([&] { hipLaunchKernelGGL((k_warp_t<2>), dim3(grid), dim3(256), 0, 0, a); }, "folded bytes mad24");
    check("folded bytes mad24");
    timeit([&] { hipLaunchKernelGGL((k_warp_t<4>), dim3(grid), dim3(256), 0, 0, a); }, "folded bytes row-ILP");
    check("folded bytes row-ILP");
    timeit([&] { hipLaunchKernelGGL((k_warp_t<6>), dim3(grid), dim3(256), 0, 0, a); }, "row-ILP + 16B staging");
    check("row-ILP + 16B staging");
    timeit([&] { hipLaunchKernelGGL((k_warp_x<0, false>), dim3(grid), dim3(256), 0, 0, a); }, "reg-staged bytes");
    check("reg-staged bytes");
    timeit([&] { hipLaunchKernelGGL((k_warp_x<0, true>), dim3(grid), dim3(256), 0, 0, a); }, "reg-pipelined bytes");
    check("reg-pipelined bytes");
    timeit([&] { hipLaunchKernelGGL((k_warp_x<1, false>), dim3(grid), dim3(256), 0, 0, a); }, "reg-staged dot4");
    check("reg-staged dot4");
    timeit([&] { hipLaunchKernelGGL((k_warp_x<1, true>), dim3(grid), dim3(256), 0, 0, a); }, "reg-pipelined dot4");
    check("reg-pipelined dot4");
    for (int g : {1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "reg-pipelined dot4 g%d", g);
        timeit([&] { hipLaunchKernelGGL((k_warp_x<1, true>), dim3(g), dim3(256), 0, 0, a); }, nm);
        check(nm);
    }
    printf("tiles %ld grid %d\n", tiles, grid);
    return 0;
}
