// Window-load rate of the pose-cell kernels' load phase: one block per CU stages the
// (tx + 2h) x (ty + 2h) cells around its tile, all TH layers (theta-fastest, C order
// (x, y, th) as the column and halo forms keep P), into LDS -- by LDS-DMA
// (global_load_lds_dwordx4, one 16-byte piece per lane) or through VGPRs
// (global_load_dwordx4, then ds_write_b128) -- right after a kernel that rewrote every
// tile of P (as the step before does).  Prints the median block span of the load and
// the per-CU rate, by mode, waves per block and window.
// usage: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_window.hip -o /tmp/ubw && /tmp/ubw
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int X = 128, Y = 128, TH = 72, U = TH / 4;
constexpr int LDS_BYTES = 150 * 1024;

__device__ inline int xcd_tile(int b, int nb) { return (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3); }

__global__ void k_write(float* P, int tx, int ty, float v) {
    const int cgy = Y / ty, tile = xcd_tile(blockIdx.x, gridDim.x);
    const int x0 = (tile / cgy) * tx, y0 = (tile % cgy) * ty;
    for (int i = threadIdx.x; i < tx * ty * U; i += blockDim.x) {
        const int u = i % U, c = i / U, cy = c % ty, cx = c / ty;
        float4* d = reinterpret_cast<float4*>(P + ((size_t)(x0 + cx) * Y + y0 + cy) * TH) + u;
        *d = make_float4(v, v + 1, v + 2, v + 3);
    }
}

template <int MODE, int K, int ADDR>
__global__ __launch_bounds__(1024) void k_read(const float* P, int tx, int ty, int h, unsigned long long* span,
                                               float* sink) {
    extern __shared__ uint4 lds[];
    const unsigned long long t0 = wall_clock64();
    const int cgy = Y / ty, tile = ADDR == 2 ? 0 : xcd_tile(blockIdx.x, gridDim.x);
    const int x0 = (tile / cgy) * tx - h, y0 = (tile % cgy) * ty - h;
    const int wy = ty + 2 * h, wx = tx + 2 * h, np = wx * wy * U;
    const uint4* lin = reinterpret_cast<const uint4*>(P) + (size_t)tile * np % ((size_t)X * Y * U - np);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    auto src = [&](int p) {
        if constexpr (ADDR == 1) return lin + p;
        const int u = p % U, c = p / U, cy = c % wy, cx = c / wy;
        const int gx = (x0 + cx + X) % X, gy = (y0 + cy + Y) % Y;
        return reinterpret_cast<const uint4*>(P + ((size_t)gx * Y + gy) * TH) + u;
    };
    if constexpr (MODE == 0 && ADDR == 3) {
        // incremental addressing: the lane's (cell column, cell row, unit) advanced by
        // the per-instruction stride with carries, no division per piece
        const int S = nw * 64, dc = S / U, du = S - dc * U, dcx = dc / wy, dcy = dc - dcx * wy;
        int p = wave * 64 + lane, u = p % U, c = p / U, cx = c / wy, cy = c - cx * wy;
        for (int i0 = wave * 64; i0 < np; i0 += S) {
            int gx = x0 + cx, gy = y0 + cy;
            gx += gx < 0 ? X : (gx >= X ? -X : 0);
            gy += gy < 0 ? Y : (gy >= Y ? -Y : 0);
            const uint4* a = i0 + lane < np ? reinterpret_cast<const uint4*>(P + ((size_t)gx * Y + gy) * TH) + u
                                            : reinterpret_cast<const uint4*>(P);
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)a,
                                             (__attribute__((address_space(3))) void*)(lds + i0), 16, 0, 0);
            u += du;
            cy += dcy;
            cx += dcx;
            if (u >= U) { u -= U; ++cy; }
            if (cy >= wy) { cy -= wy; ++cx; }
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    } else if constexpr (MODE == 0) {
        for (int i0 = wave * 64; i0 < np; i0 += nw * 64)
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)src(min(i0 + lane, np - 1)),
                                             (__attribute__((address_space(3))) void*)(lds + i0), 16, 0, 0);
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    } else {
        uint4 r[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int p = (k * nw + wave) * 64 + lane;
            if (p < np) r[k] = *src(p);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int p = (k * nw + wave) * 64 + lane;
            if (p < np) lds[p] = r[k];
        }
    }
    __syncthreads();
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) span[blockIdx.x] = t1 - t0;
    // keep the loads live
    const uint4 q = lds[(threadIdx.x * 37) % np];
    if (q.x == 0x7fffffffu) sink[threadIdx.x] = 1.f;
}

template <int MODE, int K, int ADDR = 0>
void run(float* P, unsigned long long* span, float* sink, int tx, int ty, int h, int nw, int cus) {
    const int nb = (X / tx) * (Y / ty);
    const int np = (tx + 2 * h) * (ty + 2 * h) * U;
    const size_t lds = (size_t)np * 16;
    if (lds > LDS_BYTES) return;
    if (MODE == 1 && K * nw * 64 < np) return;   // (the register form holds K pieces per lane)
    if (MODE == 1 && K * nw * 64 >= 2 * np && K > 1) return;
    hipFuncSetAttribute((const void*)k_read<MODE, K, ADDR>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    std::vector<unsigned long long> all;
    std::vector<unsigned long long> hs(nb);
    for (int it = 0; it < 60; ++it) {
        hipLaunchKernelGGL(k_write, dim3(nb), dim3(256), 0, 0, P, tx, ty, (float)it);
        hipLaunchKernelGGL((k_read<MODE, K, ADDR>), dim3(nb), dim3(64 * nw), lds, 0, P, tx, ty, h, span, sink);
        if (it >= 10) {
            hipMemcpy(hs.data(), span, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost);
            all.insert(all.end(), hs.begin(), hs.end());
        }
    }
    hipDeviceSynchronize();
    std::sort(all.begin(), all.end());
    const double med = all[all.size() / 2] / 100.0, p90 = all[all.size() * 9 / 10] / 100.0;   // 100 MHz -> us
    printf("%-6s %s K=%d tile %2dx%-2d halo %d waves %2d: %6.1f KB/block, median %.2f us (p90 %.2f): %5.1f GB/s per CU, "
           "%5.2f TB/s chip over %d blocks\n",
           MODE == 0 ? "lds-dma" : "vgpr", ADDR == 0 ? "window" : ADDR == 1 ? "linear" : ADDR == 2 ? "tile-0" : "win-inc", K, tx, ty, h, nw, lds / 1024.0, med, p90, lds / (med * 1e3),
           lds * (double)std::min(nb, cus) / (med * 1e6), nb);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* P;
    unsigned long long* span;
    float* sink;
    hipMalloc(&P, sizeof(float) * X * Y * TH);
    hipMalloc(&span, sizeof(unsigned long long) * 4096);
    hipMalloc(&sink, sizeof(float) * 1024);
    hipMemset(P, 0, sizeof(float) * X * Y * TH);
    const int tiles[][3] = {{8, 8, 3}, {8, 8, 6}};
    for (auto& t : tiles)
        for (int nw : {8, 12, 16}) {
            run<0, 1, 0>(P, span, sink, t[0], t[1], t[2], nw, cus);
            run<0, 1, 1>(P, span, sink, t[0], t[1], t[2], nw, cus);
            run<0, 1, 2>(P, span, sink, t[0], t[1], t[2], nw, cus);
            run<0, 1, 3>(P, span, sink, t[0], t[1], t[2], nw, cus);
            run<1, 4, 1>(P, span, sink, t[0], t[1], t[2], nw, cus);
            run<1, 8, 1>(P, span, sink, t[0], t[1], t[2], nw, cus);
            run<1, 16, 1>(P, span, sink, t[0], t[1], t[2], nw, cus);
        }
    printf("done\n");
    return 0;
}
