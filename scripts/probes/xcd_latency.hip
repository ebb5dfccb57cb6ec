// Cross-workgroup hand-off latency on MI355X (gfx950): what one hop of the per-step filter's
// granule exchange (csrc/rollout.hip sn_put / sn_get: relaxed agent-scope 8-byte atomics) costs.
//
//   (1) dependent agent-scope loads of one granule by one lane (load round trip)
//   (2) ping-pong between two workgroups: A stores tag k, B polls until it sees k and stores k
//       back, A polls ... (one-way hop = store visible + poll), for a pair on different XCDs
//       (blocks 0 / 1: placement is round-robin over the 8 XCDs) and on the same XCD (3 / 11)
//
// Times are s_memrealtime ticks (100 MHz).  Every spin is bounded: a missing peer ends the run.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/xcd_latency.hip -o scripts/probes/xcd_latency
//   ./scripts/probes/xcd_latency
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned long long u64;

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__device__ __forceinline__ void put(u64* g, u64 v) {
  __hip_atomic_store(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 get(const u64* g) {
  return __hip_atomic_load(const_cast<u64*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr unsigned SPIN_MAX = 1u << 22;

// out[0..3]: load-chase ticks, cross-XCD ping-pong ticks, same-XCD ping-pong ticks, error flag
__global__ void probe(u64* slots, u64* out, int n) {
  const int b = blockIdx.x;
  if (threadIdx.x != 0) return;
  if (b == 2) {   // (1) n dependent loads: the address of load i+1 depends on load i's value
    u64 idx = 0;
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < n; ++i) idx = get(slots + 64 + (idx & 1));
    const u64 t1 = __builtin_amdgcn_s_memrealtime();
    out[0] = t1 - t0 + (idx & 2);   // (idx is 0: keeps the chain live)
    return;
  }
  // (2) ping-pong pairs: blocks 0 / 1 on different XCDs, blocks 3 / 11 on the same XCD (3)
  int role = -1, pair = -1;
  if (b == 0) { role = 0; pair = 0; }
  if (b == 1) { role = 1; pair = 0; }
  if (b == 3) { role = 0; pair = 1; }
  if (b == 11) { role = 1; pair = 1; }
  if (role < 0) return;
  u64* ping = slots + 128 * pair;        // A -> B
  u64* pong = slots + 128 * pair + 32;   // B -> A (a different 256-byte line)
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  for (int k = 1; k <= n; ++k) {
    if (role == 0) {
      put(ping, (u64)k);
      unsigned s = 0;
      while (get(pong) != (u64)k)
        if (++s > SPIN_MAX) { out[3] = 1; return; }
    } else {
      unsigned s = 0;
      while (get(ping) != (u64)k)
        if (++s > SPIN_MAX) { out[3] = 1; return; }
      put(pong, (u64)k);
    }
  }
  const u64 t1 = __builtin_amdgcn_s_memrealtime();
  if (role == 0) out[1 + pair] = t1 - t0;
}

int main() {
  const int n = 2000;
  u64 *slots, *out;
  CK(hipMalloc(&slots, 4096 * sizeof(u64)));
  CK(hipMalloc(&out, 4 * sizeof(u64)));
  CK(hipMemset(slots, 0, 4096 * sizeof(u64)));
  CK(hipMemset(out, 0, 4 * sizeof(u64)));
  hipLaunchKernelGGL(probe, dim3(16), dim3(64), 0, 0, slots, out, n);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  u64 h[4];
  CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
  if (h[3]) {
    printf("{\"error\": \"a peer never answered\"}\n");
    return 2;
  }
  const double tick_ns = 10.0;
  printf("{\"agent_scope_load_round_trip_ns\": %.1f, \"cross_xcd_one_way_hop_ns\": %.1f, "
         "\"same_xcd_one_way_hop_ns\": %.1f, \"iterations\": %d}\n",
         h[0] * tick_ns / n, h[1] * tick_ns / (2.0 * n), h[2] * tick_ns / (2.0 * n), n);
  CK(hipFree(slots));
  CK(hipFree(out));
  return 0;
}
