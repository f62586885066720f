/* Sanitizer fuzz of the device-plan builder (csrc/host/devplan.c) and its pairing proof
 * (calls.c), CPU only: random shapes (P, A, -d aligned and not, -c, method 1-20, G GPUs), every
 * plan form -- direct, two-sided, one-sided, relay, coalesced relay (uniform cuts, weighted splits,
 * large-piece calls) -- built for every GPU, proven to pair (xg_devplans_match), freed.  Built with
 * all host sources by tests/test_calls_fuzz.py under -fsanitize=address,undefined: out-of-bounds
 * piece bookkeeping, uninitialised shares or leaks in the builders abort the run. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "xg_sched.h"

static unsigned long long rng = 0x9E3779B97F4A7C15ull;
static int rnd(int n)
{
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (int)(rng % (unsigned long long)n);
}

int main(int argc, char **argv)
{
    static const int forms[][2] = {{0, -1}, {4 << 20, 0}, {4 << 20, 1}, {0, XG_RELAY}, {0, XG_RELAY_COALESCED}};
    static const long long sizes[] = {24, 4096, 65536 + 48, (1 << 20), (1 << 20) + 3, (2 << 20) + 5, (12 << 20) + 3};
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    int it, built = 0, refused = 0, relayed = 0;
    for (it = 0; it < iters; ++it) {
        const int P = 2 + rnd(39), A = 1 + rnd(P < 16 ? P : 16), G = 1 + rnd(P < 8 ? P : 8);
        const long long d = sizes[rnd(7)];
        const int cs[] = {1, 2, 3, 8, 200000000}, c = cs[rnd(5)], m = 1 + rnd(20);
        int rl[64], f, g;
        char err[512];
        xg_sched *s;
        if (xg_aggregator_list(P, A, 1, 1, rl) != 0) { fprintf(stderr, "aggregator list P%d A%d\n", P, A); return 1; }
        s = xg_sched_build(m, P, A, d, c, rl, 1, 1, 0, XG_MPICH_EAGER_LIMIT, err, sizeof err);
        if (!s) { ++refused; continue; }      /* a schedule MPI deadlocks on (m6) */
        for (f = 0; f < 5; ++f) {
            xg_devplan *plans[8];
            for (g = 0; g < G; ++g) {
                plans[g] = xg_devplan_build_form(s, G, g, forms[f][0], 0, forms[f][1]);
                if (!plans[g]) { fprintf(stderr, "plan failed P%d A%d d%lld c%d m%d G%d form %d\n", P, A, d, c, m, G, f); return 1; }
            }
            if (xg_devplans_match((const xg_devplan *const *)plans, G, 0, NULL, 0, err, sizeof err) < 0) {
                fprintf(stderr, "pairing: %s (P%d A%d d%lld c%d m%d G%d form %d)\n", err, P, A, d, c, m, G, f);
                return 1;
            }
            for (g = 0; g < G; ++g) {
                int st;
                for (st = 0; f >= 3 && g == 0 && st < plans[g]->nsteps; ++st) {
                    const xg_stepplan *sp = &plans[g]->steps[st];
                    int i;
                    for (i = 0; i < sp->p2p_count; ++i) relayed += plans[g]->p2p[sp->p2p_begin + i].group == 1;
                }
                xg_devplan_free(plans[g]);
            }
            ++built;
        }
        xg_sched_free(s);
    }
    printf("ok after %d jobs: %d plan sets built, %d refused, %d second-group calls on GPU 0\n", iters, built, refused,
           relayed);
    return 0;
}
