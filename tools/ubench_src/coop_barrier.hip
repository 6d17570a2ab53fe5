// Cost of a grid-wide barrier on MI355X: cooperative-groups grid.sync()
// against an atomic sense-counter barrier, for several grid sizes.
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>
#include <cstdio>
namespace cg = cooperative_groups;

__global__ void k_cg(int iters, unsigned* sink) {
  cg::grid_group g = cg::this_grid();
  for (int i = 0; i < iters; ++i) g.sync();
  if (blockIdx.x == 0 && threadIdx.x == 0) sink[0] = iters;
}

__device__ __forceinline__ void my_barrier(unsigned* bar, unsigned nb) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned gen = __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_thread_fence(__ATOMIC_RELEASE);
    if (atomicAdd(&bar[0], 1u) == nb - 1) {
      __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&bar[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) __builtin_amdgcn_s_sleep(1);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
}

__global__ void k_my(int iters, unsigned* bar) {
  for (int i = 0; i < iters; ++i) my_barrier(bar, gridDim.x);
}

// two-level arrival: groups of 16 blocks count on their own word (separate
// 128-B lines); the last arrival of a group bumps the top counter; everyone
// waits on the generation word.
__device__ __forceinline__ void tree_barrier(unsigned* bar, unsigned nb) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned ngroups = (nb + 15) / 16;
    const unsigned grp = blockIdx.x / 16;
    const unsigned gsize = min(16u, nb - grp * 16);
    unsigned* gen = bar;
    unsigned* top = bar + 32;
    unsigned* gc = bar + 64 + grp * 32;
    const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_thread_fence(__ATOMIC_RELEASE);
    if (atomicAdd(gc, 1u) == gsize - 1) {
      __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (atomicAdd(top, 1u) == ngroups - 1) {
        __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) __builtin_amdgcn_s_sleep(1);
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
}

__global__ void k_tree(int iters, unsigned* bar) {
  for (int i = 0; i < iters; ++i) tree_barrier(bar, gridDim.x);
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  unsigned *d, *bar;
  (void)hipMalloc(&d, 64);
  (void)hipMalloc(&bar, 64 * 1024);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int iters = 100;
  for (int blocks : {64, 128, 256, 512}) {
    for (int kind = 0; kind < 3; ++kind) {
      float best = 1e9f;
      for (int rep = 0; rep < 5; ++rep) {
        int it = iters;
        (void)hipMemset(bar, 0, 64 * 1024);
        (void)hipDeviceSynchronize();
        void* args0[] = {&it, kind == 0 ? (void*)&d : (void*)&bar};
        (void)hipEventRecord(a, 0);
        hipError_t e;
        if (kind == 0) e = hipLaunchCooperativeKernel((void*)k_cg, dim3(blocks), dim3(256), args0, 0, 0);
        else if (kind == 1) e = hipLaunchCooperativeKernel((void*)k_my, dim3(blocks), dim3(256), args0, 0, 0);
        else e = hipLaunchCooperativeKernel((void*)k_tree, dim3(blocks), dim3(256), args0, 0, 0);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        if (e != hipSuccess) { printf("launch error %s\n", hipGetErrorString(e)); return 1; }
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("blocks %4d %-10s %7.2f us per barrier\n", blocks, kind == 2 ? "tree16" : kind ? "atomic" : "cg::grid", best * 1e3f / iters);
    }
  }
  return 0;
}
