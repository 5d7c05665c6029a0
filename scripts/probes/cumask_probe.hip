// Which CUs does a stream created with hipExtStreamCreateWithCUMask run on?
// Each workgroup records its hardware location (XCC, SE, SH, CU from the
// HW_ID / XCC_ID registers); the host counts distinct CUs per mask pattern.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <set>
#include <vector>

__global__ void where(unsigned* out, int spin) {
  unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID, 32 bits
  unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID, 16 bits
  long t0 = clock64();
  while (clock64() - t0 < spin) {
  }
  if (threadIdx.x == 0) out[blockIdx.x] = (xcc & 0xf) << 16 | ((hw >> 8) & 0xf) | ((hw >> 12) & 1) << 4 | ((hw >> 13) & 7) << 5;
}

static int run(const char* name, std::vector<uint32_t> mask, int nwg) {
  hipStream_t s;
  if (mask.empty()) {
    if (hipStreamCreate(&s) != hipSuccess) return 1;
  } else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
    printf("%s: create failed\n", name);
    return 1;
  }
  unsigned* d;
  hipMalloc(&d, nwg * 4);
  where<<<nwg, 64, 0, s>>>(d, 200000);
  hipStreamSynchronize(s);
  std::vector<unsigned> h(nwg);
  hipMemcpy(h.data(), d, nwg * 4, hipMemcpyDeviceToHost);
  std::set<unsigned> cus, xccs;
  for (unsigned v : h) {
    cus.insert(v);
    xccs.insert(v >> 16);
  }
  printf("%-28s distinct CUs %3zu  XCCs %zu\n", name, cus.size(), xccs.size());
  hipFree(d);
  hipStreamDestroy(s);
  return 0;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int words = (ncu + 31) / 32;
  const int nwg = ncu * 8;
  printf("device CUs %d\n", ncu);
  run("no mask", {}, nwg);
  std::vector<uint32_t> all(words, 0xffffffffu);
  run("all bits", all, nwg);
  for (int r : {8, 16, 32}) {
    // spread: k*(ncu/r) + (k % 8) (runtime.spread_cus)
    std::vector<uint32_t> m = all;
    const int step = ncu / r;
    for (int k = 0; k < r; ++k) {
      const int i = (k * step + (k % 8)) % ncu;
      m[i / 32] &= ~(1u << (i % 32));
    }
    char nm[64];
    snprintf(nm, sizeof nm, "spread minus %d", r);
    run(nm, m, nwg);
    // the first r bits
    m = all;
    for (int i = 0; i < r; ++i) m[i / 32] &= ~(1u << (i % 32));
    snprintf(nm, sizeof nm, "first %d bits off", r);
    run(nm, m, nwg);
    // the last r bits
    m = all;
    for (int i = ncu - r; i < ncu; ++i) m[i / 32] &= ~(1u << (i % 32));
    snprintf(nm, sizeof nm, "last %d bits off", r);
    run(nm, m, nwg);
  }
  // only 32 bits on (one word)
  std::vector<uint32_t> one(words, 0);
  one[0] = 0xffffffffu;
  run("only word 0 on", one, nwg);
  return 0;
}
