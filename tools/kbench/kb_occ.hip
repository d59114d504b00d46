// kb_occ.hip -- why did hipOccupancyMaxActiveBlocksPerMultiprocessor return
// 0 with hipSuccess for the one-launch step's kernels (What's
// weak #3)?  And what does it take to make co-waiting grids safe?
//
//   1. The query against a kernel's attributes: 1,024-thread workgroups with
//      a forced VGPR count (an asm clobber of v<N-1>), dynamic LDS from 0 to
//      160 KiB, before and after hipFuncSetAttribute(MaxDynamicSharedMemory).
//   2. A rendezvous kernel (every workgroup arrives on a counter, then waits
//      for all of them; bounded by the 100 MHz clock): one launch of 256
//      workgroups x 1,024 threads x 144.5 KiB alone, plainly and through
//      hipLaunchCooperativeKernel (accepted? cost per launch?).
//   3. Two streams launching that kernel at once (the hazard: each grid holds
//      part of the CUs), plainly, cooperatively, and serialised by an event
//      chain between the streams.
//   hipcc --offload-arch=gfx950 -O3 -o kb_occ kb_occ.hip && ./kb_occ
//   (-DKB_SHARED -shared -fPIC -o kb_occ.so: kb_occ_main() for a process that
//   imported torch first, i.e. runs on torch's bundled HIP runtime)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

#define CLOBBER_V(n) asm volatile("" ::: "v" #n)

template <int V>
__global__ __launch_bounds__(1024) void k_regs(float *out) {
    extern __shared__ float lds[];
    if (V >= 110) CLOBBER_V(109);
    if (V >= 128) CLOBBER_V(127);
    if (V >= 200) CLOBBER_V(199);
    if (threadIdx.x == 0 && out) out[blockIdx.x] = lds[0];
}

// Every workgroup adds 1 to *cnt, then waits until it reaches `target`
// (this launch's grid on top of the earlier launches'); a wait longer than
// `tmo` ticks of the 100 MHz clock gives up and counts itself in *late.
__global__ __launch_bounds__(1024) void k_rendezvous(unsigned *cnt, unsigned target, unsigned *late, uint64_t tmo) {
    extern __shared__ float lds[];
    CLOBBER_V(109);
    if (threadIdx.x == 0) {
        lds[0] = 1.0f;
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > tmo) {
                __hip_atomic_fetch_add(late, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}

template <typename F>
void query(const char *name, F fn, int threads) {
    hipFuncAttributes a{};
    CK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(fn)));
    printf("%-14s regs %3d static LDS %zu maxThreads %d maxDynLDS %d |", name, a.numRegs, a.sharedSizeBytes,
           a.maxThreadsPerBlock, a.maxDynamicSharedSizeBytes);
    const size_t sizes[] = {0, 16384, 49664, 65536, 65537, 98304, 147968, 157248, 163840};
    for (size_t s : sizes) {
        int n = -1;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void *>(fn), threads, s);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            printf(" %zu:err%d", s, (int)e);
        } else
            printf(" %zu:%d", s, n);
    }
    printf("\n");
}

#ifdef KB_SHARED
extern "C" int kb_occ_main() {
#else
int main() {
#endif
    int rtv = 0;
    CK(hipRuntimeGetVersion(&rtv));
    printf("HIP runtime version %d\n", rtv);
    int dev = 0, ncu = 0, lds_cu = 0, lds_blk = 0, optin = 0, clk = 0, coop = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
    CK(hipDeviceGetAttribute(&lds_blk, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
    CK(hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev));
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeWallClockRate, dev));
    CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    int regs_blk = 0, regs_cu = 0;
    CK(hipDeviceGetAttribute(&regs_blk, hipDeviceAttributeMaxRegistersPerBlock, dev));
    CK(hipDeviceGetAttribute(&regs_cu, hipDeviceAttributeMaxRegistersPerMultiprocessor, dev));
    printf("CUs %d  LDS/CU %d  LDS/block %d  optin %d  regs/block %d regs/CU %d  wallclock %d kHz  coop %d\n", ncu,
           lds_cu, lds_blk, optin, regs_blk, regs_cu, clk, coop);

    printf("-- occupancy per CU at 1,024 threads, by dynamic LDS (bytes:blocks) --\n");
    query("regs~0", k_regs<0>, 1024);
    query("regs>=110", k_regs<110>, 1024);
    query("regs>=128", k_regs<128>, 1024);
    query("regs>=200/512t", k_regs<200>, 512);
    query("rendezvous", k_rendezvous, 1024);
    for (int lim : {65536, 163840}) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k_regs<110>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lim);
        printf("hipFuncSetAttribute(MaxDynamicSharedMemorySize, %d) -> %d\n", lim, (int)e);
        (void)hipGetLastError();
        query("regs>=110", k_regs<110>, 1024);
    }

    const uint64_t tmo = (uint64_t)clk * 100;  // 100 ms in ticks of clk kHz
    unsigned *cnt = nullptr, *late = nullptr;
    CK(hipMalloc(&cnt, 64 * sizeof(unsigned)));
    CK(hipMalloc(&late, 64 * sizeof(unsigned)));
    const size_t lds = 147968;
    const unsigned grid = (unsigned)ncu;
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    auto reset = [&]() {
        CK(hipMemset(cnt, 0, 64 * sizeof(unsigned)));
        CK(hipMemset(late, 0, 64 * sizeof(unsigned)));
        CK(hipDeviceSynchronize());
    };
    auto lates = [&](int i) {
        unsigned h[64];
        CK(hipMemcpy(h, late, sizeof(h), hipMemcpyDeviceToHost));
        return h[i];
    };
    auto launch = [&](bool cooperative, hipStream_t s, unsigned *c, unsigned target, unsigned *l) -> hipError_t {
        if (!cooperative) {
            hipLaunchKernelGGL(k_rendezvous, dim3(grid), dim3(1024), lds, s, c, target, l, tmo);
            return hipGetLastError();
        }
        void *args[] = {&c, &target, &l, (void *)&tmo};
        return hipLaunchCooperativeKernel(reinterpret_cast<const void *>(k_rendezvous), dim3(grid), dim3(1024), args,
                                          (unsigned)lds, s);
    };

    printf("-- one stream: %u workgroups x 1,024 threads x %zu B LDS, 200 launches --\n", grid, lds);
    for (int coopl = 0; coopl < 2; ++coopl) {
        reset();
        hipError_t e = launch(coopl, s0, cnt, grid, late);
        if (e != hipSuccess) {
            printf("%s launch: error %d (%s)\n", coopl ? "cooperative" : "plain", (int)e, hipGetErrorString(e));
            (void)hipGetLastError();
            continue;
        }
        CK(hipStreamSynchronize(s0));
        reset();
        CK(hipEventRecord(e0, s0));
        for (unsigned i = 0; i < 200; ++i) CK(launch(coopl, s0, cnt, (i + 1) * grid, late));
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%s: %.2f us per launch, late waits %u\n", coopl ? "cooperative" : "plain", ms * 1000 / 200, lates(0));
    }
    // too large a grid for a cooperative launch
    {
        unsigned g2 = grid * 2;
        void *args[] = {&cnt, &g2, &late, (void *)&tmo};
        hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(k_rendezvous), dim3(g2), dim3(1024),
                                                  args, (unsigned)lds, s0);
        printf("cooperative launch of %u workgroups: %d (%s)\n", g2, (int)e, hipGetErrorString(e));
        (void)hipGetLastError();
        CK(hipDeviceSynchronize());
    }

    printf("-- two streams at once, 50 launches each --\n");
    for (int mode = 0; mode < 3; ++mode) {  // 0 plain, 1 cooperative, 2 plain + event chain
        reset();
        hipEvent_t chain = nullptr;
        std::vector<hipEvent_t> evs;
        bool ok = true;
        for (unsigned i = 0; i < 50 && ok; ++i)
            for (int k = 0; k < 2 && ok; ++k) {
                hipStream_t s = k ? s1 : s0;
                if (mode == 2 && chain) CK(hipStreamWaitEvent(s, chain, 0));
                hipError_t e = launch(mode == 1, s, cnt + 16 * k, (i + 1) * grid, late + 16 * k);
                if (e != hipSuccess) {
                    printf("mode %d: launch error %d (%s)\n", mode, (int)e, hipGetErrorString(e));
                    (void)hipGetLastError();
                    ok = false;
                }
                if (mode == 2) {
                    hipEvent_t ev;
                    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                    CK(hipEventRecord(ev, s));
                    evs.push_back(ev);
                    chain = ev;
                }
            }
        CK(hipDeviceSynchronize());
        for (hipEvent_t ev : evs) CK(hipEventDestroy(ev));
        printf("%s: late waits stream0 %u stream1 %u\n",
               mode == 0 ? "plain" : mode == 1 ? "cooperative" : "plain+event chain", lates(0), lates(16));
    }
    CK(hipFree(cnt));
    CK(hipFree(late));
    return 0;
}
