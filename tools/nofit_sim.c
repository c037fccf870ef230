/* Sequential FFD of BASELINE config 3 on the CPU (oracle generator and order): rejections,
 * how many an exact capacity-only summary of all nodes would catch at their turn, and how far
 * placements land behind the frontier.  gcc -O2 -I oracle -o /tmp/nofit_sim tools/nofit_sim.c
 * oracle/fp_oracle.c -lm  (about 5 minutes). */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include "fp_oracle.h"
int main(void) {
  const uint32_t C = 1000000, N = 100000;
  uint64_t sd = fpo_scenario_seed(0x5EED0003ull, 0);
  uint32_t *cpu = malloc(4*C), *mem = malloc(4*C), *req = malloc(4*C), *conf = malloc(4*C), *ord = malloc(4*C);
  uint32_t *cf = malloc(4*N), *mf = malloc(4*N), *lab = malloc(4*N), *cu = malloc(4*N); uint8_t *sc = malloc(N);
  fpo_gen_containers(sd, C, 7, cpu, mem, req, conf);
  fpo_gen_nodes(sd, N, 7, cf, mf, lab, cu, sc);
  fpo_ffd_order(C, cpu, mem, ord);
  uint64_t visits = 0, nofit = 0, det_cap = 0, det_cap_all = 0; uint32_t front = 0;
  uint64_t sum_behind = 0, placed = 0;
  uint32_t first_nofit_k = 0xFFFFFFFF;
  for (uint32_t k = 0; k < C; ++k) {
    uint32_t j = ord[k]; uint32_t c = cpu[j], m = mem[j], r = req[j], f = conf[j];
    uint32_t n;
    for (n = 0; n < N; ++n)
      if (sc[n] && cf[n] >= c && mf[n] >= m && (lab[n] & r) == r && (cu[n] & f) == 0) break;
    if (n < N) {
      cf[n] -= c; mf[n] -= m; cu[n] |= f; visits += n / 64 + 1; placed++;
      if (n / 64 > front) front = n / 64;
      sum_behind += front - n / 64;
    } else {
      nofit++; visits += (N + 63) / 64;
      if (first_nofit_k == 0xFFFFFFFF) first_nofit_k = k;
      int any = 0;
      for (uint32_t q = 0; q < N; ++q) if (sc[q] && cf[q] >= c && mf[q] >= m) { any = 1; break; }
      if (!any) det_cap++;
    }
  }
  printf("placed %llu nofit %llu visits(groups) %llu (%.1f per container)\n", (unsigned long long)placed,
         (unsigned long long)nofit, (unsigned long long)visits, (double)visits / C);
  printf("nofit detectable by exact capacity-only summary: %llu (%.1f%%), first nofit at k=%u\n",
         (unsigned long long)det_cap, 100.0 * det_cap / nofit, first_nofit_k);
  printf("avg groups behind frontier of placements: %.1f, final frontier %u\n", (double)sum_behind / placed, front);
  return 0;
}
