/* Critical path of the exact group pipeline on BASELINE config 3 (CPU model, diagnostics only).
 *
 * Sequential FFD (oracle generator and order) on GW-node groups.  Group j handles, in FFD
 * order, every container that reaches it (not placed in groups < j): a container that some
 * node of the group could take by cpu and mem alone (2-D capacity, current state) costs one
 * exact check (unit 1); any other costs `eps` (the batch prescan, amortised).  A group handles
 * its containers one at a time in order; container x reaches group j+1 when group j is done
 * with it:  T(j, x) = max(T(j, x_prev_j), T(j-1, x)) + cost(j, x).
 * Prints the critical path (the latest T) against the total number of checks: their ratio is
 * the parallelism an exact group pipeline with unit-cost checks can reach on this input.
 *   gcc -O2 -I oracle -o /tmp/front_sim tools/front_sim.c oracle/fp_oracle.c -lm
 *   /tmp/front_sim [C N eps GW]   (config 3: 1000000 100000 0.02 64) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "fp_oracle.h"

int main(int argc, char **argv) {
    const uint32_t C = argc > 1 ? (uint32_t)atol(argv[1]) : 1000000u;
    const uint32_t N = argc > 2 ? (uint32_t)atol(argv[2]) : 100000u;
    const double eps = argc > 3 ? atof(argv[3]) : 0.02;
    const int GW = argc > 4 ? atoi(argv[4]) : 64;  /* nodes per pipeline unit */
    const uint32_t G = (N + GW - 1) / GW;
    uint64_t sd = fpo_scenario_seed(0x5EED0003ull, 0);
    uint32_t *cpu = malloc(4ull * C), *mem = malloc(4ull * C), *req = malloc(4ull * C), *conf = malloc(4ull * C),
             *ord = malloc(4ull * C);
    uint32_t *cf = malloc(4ull * G * GW), *mf = malloc(4ull * G * GW), *lab = malloc(4ull * G * GW),
             *cu = malloc(4ull * G * GW);
    uint8_t *sc = calloc(G * GW, 1);
    fpo_gen_containers(sd, C, 7, cpu, mem, req, conf);
    fpo_gen_nodes(sd, N, 7, cf, mf, lab, cu, sc);
    for (uint32_t n = 0; n < G * GW; ++n)
        if (n >= N || !sc[n]) { cf[n] = 0; mf[n] = 0; sc[n] = 0; }
    fpo_ffd_order(C, cpu, mem, ord);
    double *T = calloc(G + 1, sizeof(double));      /* group j's last finish time */
    uint32_t *gmc = malloc(4ull * G), *gmm = malloc(4ull * G);  /* per-group max cf / max mf (stale-high ok) */
    for (uint32_t g = 0; g < G; ++g) {
        gmc[g] = gmm[g] = 0;
        for (int l = 0; l < GW; ++l) {
            if (cf[g * GW + l] > gmc[g]) gmc[g] = cf[g * GW + l];
            if (mf[g * GW + l] > gmm[g]) gmm[g] = mf[g * GW + l];
        }
    }
    double checks = 0, crit = 0;
    uint64_t placed = 0, misses = 0;
    uint32_t front = 0;
    double *front_t = calloc(G + 1, sizeof(double));  /* time group j first receives a check */
    for (uint32_t k = 0; k < C; ++k) {
        const uint32_t j0 = ord[k];
        const uint32_t c = cpu[j0], m = mem[j0], r = req[j0], f = conf[j0];
        double t = 0;
        uint32_t g;
        for (g = 0; g < G; ++g) {
            int cand = 0, fit = -1;
            if (gmc[g] >= c && gmm[g] >= m) {
                uint32_t nmc = 0, nmm = 0;
                for (int l = 0; l < GW; ++l) {
                    const uint32_t n = g * GW + l;
                    if (cf[n] >= c && mf[n] >= m) {
                        cand = 1;
                        if (fit < 0 && (lab[n] & r) == r && (cu[n] & f) == 0) fit = l;
                    }
                    if (cf[n] > nmc) nmc = cf[n];
                    if (mf[n] > nmm) nmm = mf[n];
                }
                gmc[g] = nmc; gmm[g] = nmm;
            }
            const double cost = cand ? 1.0 : eps;
            t = (t > T[g] ? t : T[g]) + cost;
            T[g] = t;
            if (cand) {
                checks += 1;
                if (front_t[g] == 0) front_t[g] = t;
            }
            if (fit >= 0) {
                const uint32_t n = g * GW + (uint32_t)fit;
                cf[n] -= c; mf[n] -= m; cu[n] |= f;
                placed++;
                if (g > front) front = g;
                break;
            }
            if (cand) misses++;
        }
        if (t > crit) crit = t;
    }
    printf("C=%u N=%u groups=%u eps=%.3f: placed %llu, checks %.0f (misses %llu)\n", C, N, G, eps,
           (unsigned long long)placed, checks, (unsigned long long)misses);
    printf("critical path %.0f check units = %.3f of the checks (parallelism %.1f)\n", crit, crit / checks,
           checks / crit);
    for (uint32_t g = 0; g < G; g += G / 10) printf("  group %u first check at %.0f\n", g, front_t[g]);
    return 0;
}
