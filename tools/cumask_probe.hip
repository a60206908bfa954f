// Development probe: which (XCD, CU) do the workgroups of a CU-masked stream land on?
// Build: hipcc --offload-arch=gfx950 -O2 tools/cumask_probe.hip -o tools/cumask_probe
// Prints, for a few masks, the number of distinct CUs per XCD the workgroups used.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ void probe(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));          // HW_ID
    unsigned xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11));          // XCC_ID[3:0]
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
  // stay resident a little so the dispatcher spreads the grid
  long long t0 = clock64();
  while (clock64() - t0 < 200000) {
  }
}

static void run(const char* name, const std::vector<uint32_t>& mask) {
  hipStream_t st;
  if (mask.empty()) hipStreamCreate(&st);
  else hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size() * 32, mask.data());
  const int G = 2048;
  unsigned* d;
  hipMalloc(&d, G * 2 * sizeof(unsigned));
  hipLaunchKernelGGL(probe, dim3(G), dim3(64), 0, st, d);
  std::vector<unsigned> h(G * 2);
  hipMemcpyAsync(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost, st);
  hipStreamSynchronize(st);
  std::set<std::pair<unsigned, unsigned>> cus[8];
  for (int b = 0; b < G; ++b) {
    const unsigned hw = h[2 * b], x = h[2 * b + 1] & 7;
    // cu_id [11:8], sh_id [12], se_id [15:13]
    cus[x].insert({(hw >> 13) & 7, (hw >> 8) & 31});
  }
  printf("%-28s", name);
  int tot = 0;
  for (int x = 0; x < 8; ++x) {
    printf(" x%d:%2zu", x, cus[x].size());
    tot += (int)cus[x].size();
  }
  printf("  total %d\n", tot);
  hipFree(d);
  hipStreamDestroy(st);
}

int main() {
  int n_cu = 0;
  hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", n_cu);
  const int words = (n_cu + 31) / 32;
  run("no mask", {});
  std::vector<uint32_t> m(words, 0);
  m[0] = 0xffffffffu;
  run("bits 0..31", m);
  std::fill(m.begin(), m.end(), 0u);
  for (int i = 0; i < n_cu; i += 8) m[i / 32] |= 1u << (i % 32);
  run("bits 0,8,16,..", m);
  std::fill(m.begin(), m.end(), 0xffffffffu);
  m[0] = 0;
  run("all but bits 0..31", m);
  std::fill(m.begin(), m.end(), 0xffffffffu);
  for (int i = 0; i < n_cu; i += 8) m[i / 32] &= ~(1u << (i % 32));
  run("all but 0,8,16,..", m);
  return 0;
}
