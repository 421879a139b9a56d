// Which physical CUs does a CU-masked stream use?  For a few masks, launch many short
// work-groups on a stream created with hipExtStreamCreateWithCUMask and record each
// work-group's (XCC_ID, HW_ID) — prints the distinct CUs per XCD.  Used to choose the
// matcher / tail CU split of sod_set_cu_reserve.
// hipcc --offload-arch=gfx950 -O2 tools/cu_mask_probe.hip -o tools/cu_mask_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <set>
#include <vector>

__global__ void probe(uint32_t* out) {
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
  // stay resident a little so the dispatcher spreads the work-groups
  long t0 = clock64();
  while (clock64() - t0 < 20000) {}
}

static void run(const char* name, const std::vector<uint32_t>& mask) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data())  /* words */ != hipSuccess) {
    printf("%s: stream create failed\n", name);
    return;
  }
  const int nb = 4096;
  uint32_t* d;
  hipMalloc(&d, nb * 8);
  hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d);
  hipStreamSynchronize(s);
  std::vector<uint32_t> h(nb * 2);
  hipMemcpy(h.data(), d, nb * 8, hipMemcpyDeviceToHost);
  std::set<uint32_t> cus[16];
  for (int b = 0; b < nb; ++b) {
    const uint32_t xcc = h[2 * b] & 0xf, hw = h[2 * b + 1];
    // HW_ID: cu_id [11:8], sh_id [12], se_id [15:13]
    cus[xcc].insert((hw >> 8) & 0xff);
  }
  printf("%-28s", name);
  int tot = 0;
  for (int x = 0; x < 8; ++x) {
    printf(" x%d:%2zu", x, cus[x].size());
    tot += (int)cus[x].size();
  }
  printf("  total %d\n", tot);
  hipFree(d);
  hipStreamDestroy(s);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("CUs %d\n", p.multiProcessorCount);
  const int n = p.multiProcessorCount, words = (n + 31) / 32;
  std::vector<uint32_t> all(words, 0xffffffffu);
  run("all", all);
  std::vector<uint32_t> m(words, 0);
  for (int lo : {0, 8, 32, 248}) {
    std::fill(m.begin(), m.end(), 0u);
    for (int i = lo; i < lo + 8 && i < n; ++i) m[i / 32] |= 1u << (i % 32);
    char nm[64];
    snprintf(nm, sizeof nm, "bits %d..%d", lo, lo + 7);
    run(nm, m);
  }
  std::fill(m.begin(), m.end(), 0u);
  for (int i = 0; i < 32; ++i) m[i / 32] |= 1u << i;
  run("bits 0..31", m);
  // complement of the top 8 bits
  std::vector<uint32_t> c(all);
  for (int i = n - 8; i < n; ++i) c[i / 32] &= ~(1u << (i % 32));
  run("all but top 8 bits", c);
  // one bit at a time for the first 16: which XCD does bit i land on
  for (int i = 0; i < 16; ++i) {
    std::fill(m.begin(), m.end(), 0u);
    m[i / 32] |= 1u << (i % 32);
    char nm[64];
    snprintf(nm, sizeof nm, "bit %d", i);
    run(nm, m);
  }
  return 0;
}
