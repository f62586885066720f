/* Sanitizer fuzz of xg_calls_match (csrc/host/calls.c), CPU only: random G-GPU call lists --
 * jobs built to pair step by step, then one of them broken at random -- against a brute-force
 * restatement of RCCL's pairing.  Built and run by tests/test_calls_fuzz.py with
 * -fsanitize=address,undefined (a standalone executable: no preload needed). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "xg_sched.h"

static unsigned long long rng = 88172645463325252ull;
static int rnd(int n)
{
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (int)(rng % (unsigned long long)n);
}

#define MAXC 4096

int main(int argc, char **argv)
{
    int iters = argc > 1 ? atoi(argv[1]) : 2000, it, bad = 0, refused = 0;
    for (it = 0; it < iters; ++it) {
        int G = 1 + rnd(8), S = 1 + rnd(6), g, s, k;
        static xg_call calls[8][MAXC];
        static int32_t sb[8][16];
        int n[8] = {0};
        const int barrier_step = rnd(S + 1) - 1;        /* -1: none */
        const int brk = rnd(3) == 0 ? 1 + rnd(4) : 0;  /* 0: a valid job */
        for (s = 0; s < S; ++s) {
            for (g = 0; g < G; ++g) sb[g][s] = n[g];
            /* messages of step s: (src, dst, len); sends/recvs appended in message order */
            int nm = rnd(12);
            for (k = 0; k < nm; ++k) {
                int a = rnd(G), b = rnd(G);
                long long len = 16 * (1 + rnd(64));
                xg_call *c = &calls[a][n[a]++];
                memset(c, 0, sizeof *c);
                c->kind = XG_CALL_SEND; c->peer = b; c->buf = 0; c->off = 0; c->len = len;
                c = &calls[b][n[b]++];
                memset(c, 0, sizeof *c);
                c->kind = XG_CALL_RECV; c->peer = a; c->buf = 1; c->off = 0; c->len = len;
            }
            if (s == barrier_step)
                for (g = 0; g < G; ++g) {
                    xg_call *c = &calls[g][n[g]++];
                    memset(c, 0, sizeof *c);
                    c->kind = XG_CALL_BARRIER; c->peer = -1; c->buf = -1;
                }
        }
        for (g = 0; g < G; ++g) sb[g][S] = n[g];
        /* break it: drop a receive / change a length / move a barrier / corrupt a peer */
        if (brk) {
            int gg = rnd(G), found = -1;
            for (k = 0; k < n[gg]; ++k)
                if ((brk == 1 && calls[gg][k].kind == XG_CALL_RECV) || (brk == 2 && calls[gg][k].kind == XG_CALL_SEND) ||
                    (brk == 3 && calls[gg][k].kind == XG_CALL_BARRIER) || brk == 4) { found = k; break; }
            if (found < 0) continue;
            if (brk == 1) calls[gg][found].kind = XG_CALL_SEND;            /* a receive turned into a send */
            else if (brk == 2) calls[gg][found].len += 16;                 /* a length off */
            else if (brk == 3) calls[gg][found].kind = XG_CALL_SEND, calls[gg][found].peer = gg, calls[gg][found].len = 16;
            else calls[gg][found].peer = G + rnd(3);                       /* a peer out of range */
        }
        {
            const xg_call *cp[8];
            const int32_t *bp[8];
            char err[256];
            long long np;
            xg_call_pair *out;
            for (g = 0; g < G; ++g) { cp[g] = calls[g]; bp[g] = sb[g]; }
            np = xg_calls_match(G, S, cp, bp, NULL, 0, err, sizeof err);
            if (!brk && np < 0) { printf("iter %d: valid job refused: %s\n", it, err); bad++; continue; }
            if (brk && np < 0) refused++;
            if (brk && np >= 0) {
                /* a broken job may still pair only when the change kept every channel consistent */
                continue;
            }
            if (np < 0) continue;
            out = (xg_call_pair *)malloc(sizeof *out * (size_t)(np + 1));
            if (xg_calls_match(G, S, cp, bp, out, np, err, sizeof err) != np) { bad++; free(out); continue; }
            /* brute force: every pair's send and receive are in the same step, same length, ordered */
            for (k = 0; k < np; ++k) {
                const xg_call *sc = &calls[out[k].src][out[k].send_call], *rc = &calls[out[k].dst][out[k].recv_call];
                if (sc->kind != XG_CALL_SEND || rc->kind != XG_CALL_RECV || sc->peer != out[k].dst ||
                    rc->peer != out[k].src || sc->len != rc->len || (k && out[k].step < out[k - 1].step)) {
                    printf("iter %d: pair %d wrong\n", it, k);
                    bad++;
                    break;
                }
            }
            free(out);
        }
    }
    printf("%s after %d jobs (%d broken jobs refused)\n", bad || !refused ? "FAILED" : "ok", iters, refused);
    return bad != 0 || !refused;
}
