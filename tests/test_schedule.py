"""The ring planner's discrete-event model (aligned_vggt/dist/schedule.py):
hand-checked timelines, the plan space, and the BASELINE configs[3]/[4]
chunking (512 frames, chunk 16 / overlap 4 -> 42 chunks + an 8-frame tail)."""
import pytest

from aligned_vggt.dist import schedule as SC
from aligned_vggt.utils.data import generate_chunks


def _costs(**kw):
    base = dict(core={(4, 1): 10.0, (4, 2): 16.0}, dense={(4, 1): 2.0, (4, 2): 3.0}, t_align=1.0,
                t_align_alone=0.5, t_pause=1.5, t_align_ungated=3.0, t_pause_ungated=0.25, hop=0.1, gather=0.0)
    base.update(kw)
    return SC.RingCosts(**base)


def test_timeline_pauses_extend_the_running_job():
    c = _costs()
    jobs = [("core", (0,)), ("dense", (0,))]
    assert SC._timeline(jobs, [4], c, [], 1.5) == [10.0, 12.0]
    # a pause at 5 lands in the core (-> 11.5), one at 12 in the shifted dense (11.5 + 2 + 1.5)
    assert SC._timeline(jobs, [4], c, [5.0, 12.0], 1.5) == [11.5, 15.0]
    # a pause at 11 still lands in the extended core
    assert SC._timeline(jobs, [4], c, [5.0, 11.0], 1.5) == [13.0, 15.0]
    # a pause after the last job costs nothing
    assert SC._timeline(jobs, [4], c, [20.0], 1.5) == [10.0, 12.0]


def test_simulate_two_ranks_by_hand():
    """2 chunks of 4 frames on 2 ranks, one "with" job each: both encodes end
    at 12; align 0 on rank 0 (rank idle -> alone 0.5) ends 12.5; the baton hop
    0.1 -> align 1 on rank 1 12.6 .. 13.1."""
    c = _costs()
    plans = [SC.RankPlan([("enc", (0,))]), SC.RankPlan([("enc", (1,))])]
    pr = SC.simulate([4, 4], 2, plans, c)
    assert pr.align_start == [12.0, 12.6]
    assert pr.align_end == [12.5, 13.1]
    assert pr.total_ms == pytest.approx(13.1)
    # deferring the DPT: the cores end at 10, the alignments overlap the dense jobs (gated: +1.5 each)
    plans = [SC.RankPlan([("core", (0,)), ("dense", (0,))]), SC.RankPlan([("core", (1,)), ("dense", (1,))])]
    pr = SC.simulate([4, 4], 2, plans, c)
    assert pr.align_start == [10.0, 11.1]
    assert pr.rank_finish == [13.5, 13.5]
    assert pr.total_ms == pytest.approx(13.5)


def test_candidate_sizes_cover_the_run():
    assert len(SC.compositions(6, 3)) == 24
    for n in (1, 5, 6, 9, 42):
        cs = SC.candidate_sizes(n, 3)
        assert cs and all(sum(c) == n and max(c) <= 3 for c in cs), n
    assert (3,) * 14 in SC.candidate_sizes(42, 3) and (2,) + (3,) * 13 + (1,) in SC.candidate_sizes(42, 3)


def test_enqueue_order_lookahead():
    plan = SC.RankPlan(SC.make_jobs([[0], [2, 4], [6]], "lag"))
    assert plan.jobs == [("core", (0,)), ("core", (2, 4)), ("dense", (0,)), ("core", (6,)), ("dense", (2, 4)),
                         ("dense", (6,))]
    order = SC.enqueue_order(plan, [0, 2, 4, 6])
    assert order == [("job", 0), ("job", 1), ("align", (0,)), ("job", 2), ("align", (2,)), ("align", (4,)),
                     ("job", 3), ("job", 4), ("align", (6,)), ("job", 5)]


@pytest.mark.parametrize("W", [2, 4, 8])
def test_planner_beats_round4_schedule_on_configs3(W):
    """On the configs[3]/[4] chunking the planner's predicted sequence time is
    never above round 4's greedy groups of 3 (DPT inside each encode), and
    every rank's plan covers exactly its own chunks, each core before its DPT."""
    L = [len(c) for c in generate_chunks(512, "chunk_overlap", 16, 4)]
    assert len(L) == 43 and L[-1] == 8
    c = SC.DEFAULT_COSTS
    plans, pr = SC.plan_ring(L, W, c)
    leg = SC.simulate(L, W, SC.legacy_plans(L, W), c)
    assert pr.total_ms <= leg.total_ms + 1e-9
    for r, pl in enumerate(plans):
        cores = [i for k, g in pl.jobs if k in ("enc", "core") for i in g]
        assert sorted(cores) == list(range(r, 43, W))
        seen = set()
        for k, g in pl.jobs:
            if k == "dense":
                assert set(g) <= seen
            if k in ("enc", "core"):
                seen |= set(g)
        dense = [i for k, g in pl.jobs if k in ("enc", "dense") for i in g]
        assert sorted(dense) == cores
    if W == 8:
        # strictly better than round 4's plan, and never below the recurrence's own
        # bound (every alignment at its alone speed, back to back from the earliest
        # possible first core); once the alignment chain starts it is busy: its waits
        # (hops, ships, an encode not yet done) add up to under 5 % of the sequence
        assert pr.total_ms < leg.total_ms
        first_core = min(v for (fr, g), v in c.core.items() if fr == L[0])
        assert pr.total_ms >= first_core + 43 * c.t_align_alone - 1e-9
        gaps = [s - e for s, e in zip(pr.align_start[1:], pr.align_end[:-1])]
        assert sum(gaps) <= 0.05 * pr.total_ms


def test_costs_roundtrip():
    c = SC.DEFAULT_COSTS
    d = c.to_json()
    assert SC.RingCosts.from_json(d) == c


@pytest.mark.parametrize("W", [2, 4])
def test_refine_never_worse_and_keeps_ownership(W):
    """The re-plan pass after the alignment moves only accepts a better
    prediction, and its alignments still sit on valid ranks with the same
    assignment on every rank's plan (configs[3]/[4] chunking)."""
    L = [len(c) for c in generate_chunks(512, "chunk_overlap", 16, 4)]
    c = SC.DEFAULT_COSTS
    _, base = SC.plan_ring(L, W, c, refine=False)
    plans, pr = SC.plan_ring(L, W, c)
    assert pr.total_ms <= base.total_ms + 1e-9
    ar = plans[0].align_rank
    assert len(ar) == len(L) and all(0 <= a < W for a in ar)
    assert all(pl.align_rank == ar for pl in plans)
    assert SC.simulate(L, W, plans, c).total_ms == pytest.approx(pr.total_ms)


def test_held_peak_by_policy():
    gs = [[0, 1], [2, 3], [4]]
    assert SC.held_peak(SC.make_jobs(gs, "with")) == 0
    assert SC.held_peak(SC.make_jobs(gs, "lag")) == 4  # core(2,3) queued before dense(0,1)
    assert SC.held_peak(SC.make_jobs(gs, "end")) == 5


def test_planner_memory_bound_on_long_sequence():
    """the one-rank plan may pick "end" (every core result held until
    the DPT jobs at the end), whose device memory grows with the sequence.  With
    max_held the plan of a long sequence holds at most that many chunks, and an
    unbounded plan shows the bound bites (2,048 frames -> 171 chunks, one rank)."""
    lengths = [len(c) for c in generate_chunks(2048, "chunk_overlap", 16, 4)]
    assert len(lengths) == 171
    costs = SC.DEFAULT_COSTS
    free, _ = SC.plan_ring(lengths, 1, costs, 3, ("with", "lag", "end"), (False,), sweeps=1)
    assert SC.held_peak(free[0].jobs) > 12  # unbounded, the planner holds many chunks
    for bound in (3, 12):
        plans, pr = SC.plan_ring(lengths, 1, costs, 3, ("with", "lag", "end"), (False,), sweeps=1, max_held=bound)
        assert SC.held_peak(plans[0].jobs) <= bound
        covered = sorted(i for kind, g in plans[0].jobs if kind in ("enc", "core") for i in g)
        assert covered == list(range(len(lengths)))
        assert pr.total_ms >= 0.0
    # at W = 8 every rank's plan stays under the bound too
    lengths = [len(c) for c in generate_chunks(512, "chunk_overlap", 16, 4)]
    plans, _ = SC.plan_ring(lengths, 8, costs, 3, max_held=3, offload=False)
    assert all(SC.held_peak(pl.jobs) <= 3 for pl in plans)
