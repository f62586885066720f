# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
"""Per-step completion times of the README-config chains under the engine modes
(step_done from the in-kernel wall-clock stamps, anchored at the run's end):
where a run's time goes -- doorbell in, per step, tail."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as G

xg = G.load_package().xg
P, A, d, c = [int(x) for x in os.environ.get("PROBE_CFG", "32,14,2048,3").split(",")]
rl = xg.aggregator_list(P, A)
modes = {"solo_armed": {}, "solo64_armed": {"XG_SOLO_RAILS": "64"}, "solo512_armed": {"XG_SOLO_RAILS": "512"},
         "solo1_armed": {"XG_SOLO_RAILS": "1"}, "solo_norelay": {"XG_SOLO_RELAY": "0", "XG_SOLO_RAILS": "16"},
         "wg16_armed": {"XG_SOLO_WAVES": "16"}, "wg4_armed": {"XG_SOLO_WAVES": "16", "XG_SOLO_RAILS": "4"},
         "wg1_armed": {"XG_SOLO_WAVES": "16", "XG_SOLO_RAILS": "1"},
         "grid_armed": {"XG_ENGINE_SOLO": "0"}, "solo_launch": {"XG_ENGINE_ARM": "0"},
         "solo_big": {"XG_ENGINE_SOLO_MAX": "268435456", "XG_ENGINE_MAX_STEP": "268435456"},
         "solo512_big": {"XG_ENGINE_SOLO_MAX": "268435456", "XG_ENGINE_MAX_STEP": "268435456", "XG_SOLO_RAILS": "512"},
         "grid_big": {"XG_ENGINE_SOLO": "0", "XG_ENGINE_MAX_STEP": "268435456"},
         "chained": {"XG_ENGINE_MAX_STEP": "0"}}
if os.environ.get("PROBE_MODES"):
    modes = {k: v for k, v in modes.items() if k in os.environ["PROBE_MODES"].split(",")}
for name, env in modes.items():
    os.environ.update(env)
    ctx = xg.Context(0, 1, device=0)
    for k in env:
        del os.environ[k]
    for m in [int(x) for x in os.environ.get("PROBE_METHODS", "6,9,12").split(",")]:
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
        run = xg.MethodRun(ctx, s, it=0, mode=0)
        best = None
        for _ in range(7):
            done, post, wall = run.run_timed()
            if best is None or done[-1] < best[0][-1]:
                best = (done, post, wall)
        done = best[0]
        steps = [done[0]] + [b - a for a, b in zip(done, done[1:])]
        print("%-12s m%-2d steps %2d total %6.1f us  first %5.1f  mean step %5.2f  max step %5.2f  last %5.2f  post %.1f" % (
            name, m, len(done), done[-1] * 1e6, done[0] * 1e6, sum(steps[1:]) / max(1, len(steps) - 1) * 1e6,
            max(steps[1:]) * 1e6, steps[-1] * 1e6, best[1][0] * 1e6), flush=True)
        print("    steps us: " + " ".join("%.2f" % (x * 1e6) for x in steps), flush=True)
        run.close()
    ctx.close()
