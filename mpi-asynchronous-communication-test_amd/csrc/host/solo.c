/*
 * solo.c -- the solo step engine's tables (kernels.h solo_engine_kernel,
 * include/xg_sched.h xg_solo_tables): a hazard-free run of steps cut into
 * 1 KiB pieces, dealt round-robin over R rails (workgroups), and per rail laid
 * out as rows of `waves` pieces (one per wave of the rail's workgroup: 16, or
 * 1 for rails of a single wave) with the step barriers placed between them.
 *
 * A rail closes a step with a workgroup barrier only if it had pieces in it:
 * the barrier sits in front of the rail's next piece -- in that piece's row,
 * counted in the `before` field of that piece and of every later piece of the
 * row, and in the row's barrier count -- and the step it closes is listed in
 * order; a barrier in front of the rail's end is left to the kernel's closing
 * stamp.  Each barrier precedes a distinct piece, so a row holds at most
 * `waves` of them (the 5-bit `before` field).  A rail's table is padded
 * with empty pieces to an even number of chunks of XG_SOLO_K rows plus one
 * spare chunk (the kernel's double-buffered loop loads one chunk past the
 * last without a branch); the kernel stops after the rows that hold real
 * pieces (meta's last R entries), so the padding costs a table slot, not time.
 *
 * Granule G (16, 4 or 1 bytes): the unit of the offsets and lengths, i.e. the
 * alignment every transfer must have -- 16 for the 16-B loads/stores of aligned
 * segments, 4 and 1 for segment sizes that are not multiples of 16 (any -d); the
 * kernel then moves a piece with 4-B or 1-B accesses (xg_solo_tables_g).
 *
 * One-wave rails (waves = 1) use the WIDE form: a row is one piece, so the row's
 * barrier word carries the piece's length (bits 8-19) beside the barrier count
 * (bits 0-7, all of which precede the piece), and the descriptor is two 32-bit
 * offsets in granules (src | dst << 32): 4-64 GiB windows instead of 16-256 MiB.
 */
#include <stdlib.h>
#include <string.h>

#include "xg.h"
#include "xg_sched.h"

static uint64_t desc(uint64_t src, uint64_t dst, uint64_t len) { return src | (dst << 24) | (len << 48); }

int xg_solo_tables(const xg_span *xfer, const int *step_begin, int nsteps, int rails_max, int waves,
                   uint64_t src_base, uint64_t dst_base, xg_solo_shape *shape, uint64_t *descs, int *meta)
{
    return xg_solo_tables_g(xfer, step_begin, nsteps, rails_max, waves, 16, src_base, dst_base, shape, descs, meta);
}

int xg_solo_tables_g(const xg_span *xfer, const int *step_begin, int nsteps, int rails_max, int waves, int granule,
                     uint64_t src_base, uint64_t dst_base, xg_solo_shape *shape, uint64_t *descs, int *meta)
{
    if (!xfer || !step_begin || !shape || nsteps < 1 || nsteps > XG_SOLO_MAX_STEPS || rails_max < 1 ||
        rails_max > XG_SOLO_MAX_RAILS || (waves != 1 && waves != XG_SOLO_WAVES) ||
        (granule != 16 && granule != 4 && granule != 1) || (granule != 16 && waves != 1))
        return XG_EARG;
    const int nx = step_begin[nsteps];
    const int W = waves;       /* pieces per row: one per wave of a rail */
    const uint64_t G = (uint64_t)granule;
    const int bshift = XG_SOLO_BEFORE_SHIFT(granule);
    const int wide = W == 1;
    const uint64_t offmax = wide ? XG_SOLO_WIDE_OFF_MAX : XG_SOLO_OFF_MAX;
    int64_t total = 0;
    for (int i = 0; i < nx; ++i) {
        const xg_span *x = &xfer[i];
        if ((x->src | x->dst | x->len) & (G - 1)) return XG_EARG;
        if (x->len && (x->src < src_base || x->dst < dst_base || (x->src + x->len - src_base) / G > offmax ||
                       (x->dst + x->len - dst_base) / G > offmax))
            return XG_EARG;
        total += (int64_t)((x->len + XG_SOLO_PIECE - 1) / XG_SOLO_PIECE);
    }
    int64_t r = total / W;
    if (r > rails_max) r = rails_max;
    if (r < 1) r = 1;
    const int rails = (int)r;
    const int64_t chunk = (int64_t)W * XG_SOLO_K;
    const int64_t longest = (total + rails - 1) / rails;     /* round-robin: counts differ by <= 1 */
    const int64_t np = ((longest + 2 * chunk - 1) / (2 * chunk) * 2 + 1) * chunk;
    shape->rails = rails;
    shape->npieces = (int)(np > XG_SOLO_MAX_PIECES ? XG_SOLO_MAX_PIECES + 1 : np);
    shape->nrows = (int)(np / W);
    shape->nmeta = rails * (shape->nrows + 1) + rails * nsteps + rails;
    if (np > XG_SOLO_MAX_PIECES) return XG_EARG;
    if (!descs || !meta) return XG_OK;

    const int nrows = shape->nrows;
    memset(descs, 0, sizeof(uint64_t) * (size_t)rails * np);
    int *close = meta, *cstep = meta + (size_t)rails * (nrows + 1);
    memset(close, 0, sizeof(int) * (size_t)rails * (nrows + 1));
    for (int64_t i = 0; i < (int64_t)rails * nsteps; ++i) cstep[i] = -1;
    int64_t *cnt = calloc((size_t)rails, sizeof(int64_t));    /* pieces dealt to each rail */
    int *nb = calloc((size_t)rails, sizeof(int));              /* barriers placed on each rail */
    char *used = calloc((size_t)rails, 1);
    int64_t *pend = calloc((size_t)rails, sizeof(int64_t));    /* open barrier position per rail, -1 none */
    int *pstep = calloc((size_t)rails, sizeof(int));
    if (!cnt || !nb || !used || !pend || !pstep) {
        free(cnt); free(nb); free(used); free(pend); free(pstep);
        return XG_ENOMEM;
    }
    for (int q = 0; q < rails; ++q) pend[q] = -1;
    int cur = 0;
    for (int t = 0; t < nsteps; ++t) {
        memset(used, 0, (size_t)rails);
        for (int i = step_begin[t]; i < step_begin[t + 1]; ++i)
            for (uint64_t o = 0; o < xfer[i].len; o += XG_SOLO_PIECE) {
                const uint64_t len = xfer[i].len - o < XG_SOLO_PIECE ? xfer[i].len - o : XG_SOLO_PIECE;
                /* a barrier still open on this rail goes in front of this piece */
                if (pend[cur] >= 0) {
                    const int64_t at = pend[cur], row = at / W;
                    close[(size_t)cur * (nrows + 1) + row]++;
                    cstep[(size_t)cur * nsteps + nb[cur]++] = pstep[cur];
                    if (!wide)                                   /* wide: `before` = the row's count */
                        for (int64_t w = at % W; w < W; ++w)
                            descs[(size_t)cur * np + row * W + w] += 1ull << bshift;
                    pend[cur] = -1;
                }
                if (wide) {
                    close[(size_t)cur * (nrows + 1) + cnt[cur]] |= (int)((len / G) << 8);
                    descs[(size_t)cur * np + cnt[cur]++] =
                        ((xfer[i].src + o - src_base) / G) | (((xfer[i].dst + o - dst_base) / G) << 32);
                } else {
                    descs[(size_t)cur * np + cnt[cur]++] +=     /* its `before` bits may be set already */
                        desc((xfer[i].src + o - src_base) / G, (xfer[i].dst + o - dst_base) / G, len / G);
                }
                used[cur] = 1;
                cur = (cur + 1) % rails;
            }
        for (int q = 0; q < rails; ++q)
            if (used[q]) {
                pend[q] = cnt[q];
                pstep[q] = t;
            }
    }
    int *rows = cstep + (size_t)rails * nsteps;               /* rows holding real pieces */
    for (int q = 0; q < rails; ++q) rows[q] = (int)((cnt[q] + W - 1) / W);
    free(cnt); free(nb); free(used); free(pend); free(pstep);
    return XG_OK;
}

/* Step times of a solo segment from its rails' stamps (kernels.h solo_engine_kernel):
 * rail r's stamp of step t is stamps[r * stride + t], 0 where the rail closed nothing;
 * a rail with nothing in step t is done with it when it closed its previous step, so
 * its value for t is its latest nonzero stamp at or before t; step t is over when every
 * rail is: out[t] = max over rails, for t in [s0, s1). */
void xg_solo_reduce_stamps(const uint64_t *stamps, int rails, int64_t stride, int s0, int s1, uint64_t *out)
{
    for (int t = s0; t < s1; ++t) out[t] = 0;
    for (int r = 0; r < rails; ++r) {
        uint64_t carry = 0;
        for (int t = s0; t < s1; ++t) {
            const uint64_t x = stamps[(int64_t)r * stride + t];
            if (x > carry) carry = x;
            if (carry > out[t]) out[t] = carry;
        }
    }
}
