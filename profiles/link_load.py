#!/usr/bin/env python3
"""Per-step xGMI link load of BASELINE.json's 8-GPU plans (CPU only: the host plans themselves).

For every method of configs[2] (P64 A16 -d 256 KiB), configs[3] (P256 A32 -d 4 MiB) and configs[4]
(P256 A64 -d 64 MiB, -c 1..8) at G = 8, and every cross-GPU form (direct, packed one-sided,
packed two-sided, relay, coalesced relay), the calls each GPU posts (xg_devplan_step_calls: what enqueue_step hands
RCCL) are summed per directed GPU link, per step and per RCCL group of the step:

  busiest   = sum over steps and groups of the most loaded link's bytes (one direction)
  ideal     = sum over steps of the step's cross-GPU bytes / (G (G - 1)): every link equally busy
  ratio     = busiest / ideal (1.0: the plan spreads its bytes over all 56 links)
  port      = sum over steps of max over GPUs of (egress, ingress) / (G - 1): what the step's own
              traffic needs through the busiest GPU's 7 links however it is routed (an incast step
              -- every GPU sending to one -- is bound there, and the direct form already meets it)
  vs port   = busiest / port (1.0: no routing of these messages could do better)
  model_ms  = busiest / L, L = 50 GB/s per link and direction (DESIGN.md section 5's model rate; the
              N > 1 bench line measures the real one in xgmi.links)

The groups of a step run one after the other (a relay step's forwards wait for its first group),
so a step costs the sum of its groups' busiest links.  Writes the table to stdout.
Reference: pairwise partners rank ^ i (mpi_test.c:531-545) put every round of m9 / m10 on ONE link.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

L_GBPS = 50.0
FORMS = (("direct", 0, -1), ("one-sided", 4 << 20, 1), ("two-sided", 4 << 20, 0), ("relay", 0, 2),
         ("coalesced", 0, 3))
CONFIGS = ([("configs[2]", 64, 16, 256 << 10, 200000000, (5, 8)),
            ("configs[3]", 256, 32, 4 << 20, 200000000, (1, 2, 9, 10))] +
           [("configs[4] -c %d" % c, 256, 64, 64 << 20, c, (7, 11, 12)) for c in range(1, 9)])


def port_bound(s, G):
    """sum over steps of the busiest GPU's (egress, ingress) cross-GPU message bytes / (G - 1)"""
    per = {}
    for src, _ss, dst, _ds, ln, st, flags in s.messages():
        gs, gd = s.gpu_of(G, src), s.gpu_of(G, dst)
        if gs == gd or ln <= 0 or flags & 4:          # local, empty, or a TAM size message (XG_MSG_CTRL)
            continue
        e = per.setdefault(st, [[0] * G, [0] * G])
        e[0][gs] += ln
        e[1][gd] += ln
    return sum(max(max(eg), max(ig)) for eg, ig in per.values()) / (G - 1)


def link_load(xg, s, G, pack, form):
    """-> (cross-GPU message bytes, bytes posted on links, busiest-link bytes summed over steps and
    groups, ideal bytes, steps, relayed steps)"""
    views = [s.devplan(G, g, pack, 0, form) for g in range(G)]
    cross = busiest = 0
    relayed = 0
    for st in range(views[0].nsteps):
        per = {}                         # (group, src, dst) -> bytes
        for g, v in enumerate(views):
            grp = 0
            for kind, peer, _buf, _off, ln in v.calls(st):
                if kind == xg.CALL_FENCE:
                    grp += 1
                elif kind == xg.CALL_SEND and peer != g:
                    per[(grp, g, peer)] = per.get((grp, g, peer), 0) + ln
                    cross += ln          # bytes posted on links, relay forwards included
        groups = {k[0] for k in per}
        relayed += len(groups) > 1
        busiest += sum(max(b for k, b in per.items() if k[0] == q) for q in groups)
    total_msg = sum(v.remote_send_bytes for v in views)       # the messages' own cross-GPU bytes
    ideal = total_msg / (G * (G - 1))
    return total_msg, cross, busiest, ideal, views[0].nsteps, relayed


def main():
    import __graft_entry__ as GE
    xg = GE.load_package().xg
    G = 8
    print("BASELINE 8-GPU plans, link load per directed xGMI link (G = 8, 56 links); model rate %.0f GB/s per link"
          % L_GBPS)
    print("%-18s %-4s %-10s %6s %8s %12s %12s %12s %7s %10s %8s %10s" % (
        "config", "m", "form", "steps", "relayed", "cross MiB", "posted MiB", "busiest MiB", "ratio", "port MiB",
        "vs port", "model ms"))
    for name, P, A, d, c, methods in CONFIGS:
        rl = xg.aggregator_list(P, A)
        for m in methods:
            s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
            port = port_bound(s, G)
            for fname, pack, form in FORMS:
                tot, posted, busiest, ideal, nst, relayed = link_load(xg, s, G, pack, form)
                print("%-18s %-4d %-10s %6d %8d %12.0f %12.0f %12.0f %7.2f %10.0f %8.2f %10.2f"
                      % (name, m, fname, nst, relayed, tot / 2 ** 20, posted / 2 ** 20, busiest / 2 ** 20,
                         busiest / ideal if ideal else 0.0, port / 2 ** 20, busiest / port if port else 0.0,
                         busiest / (L_GBPS * 1e9) * 1e3))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
