"""Per-rank encode plans for the chunk pipeline's baton ring, and the
discrete-event model that picks them.

The reference runs its chunks strictly one after another
(training_metrics.py:643-652; featureAligned_vggt.py:84-94 threads
``context`` chunk to chunk).  ``ChunkPipeline`` splits each chunk's forward
into context-free encode work and the recurrent ``align_chunk``; chunk i is
owned by rank i mod W.  A rank's encode stream runs *jobs*:

  * ``("enc", g)``   aggregator + camera head + alignment prefix + DPT heads of
    the chunks in ``g`` as one batch (``encode_chunk``);
  * ``("core", g)``  the same without the DPT heads -- everything the
    alignment recurrence needs (``encode_chunk(..., dense=False)``);
  * ``("dense", g)`` the DPT heads of a group whose core ran earlier
    (``encode_dense``); its outputs are scaled by the chunk Sim(3) after the
    alignment (featureAligned_vggt.py:171) at the end of the sequence.

Alignment i runs on rank i mod W when chunk i's core is done and alignment
i-1 has finished on the previous rank (+ one baton hop); while it runs, the
rank's encode stream is paused by the encode gate (runtime.EncodeGate).
Grouping chunks makes each encode more efficient (6,592-row 154x518 chunks
fill the GPU poorly one at a time) but delays the first chunk of a group, and
a large group at the end of a rank's plan leaves many alignments to run after
the last encode.  ``simulate`` predicts the sequence time of a set of plans
from measured per-job costs; ``plan_ring`` searches group sizes and the DPT
placement rank by rank (coordinate descent) for the smallest predicted time.
Plans change only the order of work, never the results (tests/test_dist_pipeline.py).
"""
from __future__ import annotations

import bisect
import json
import os
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

Job = Tuple[str, Tuple[int, ...]]


@dataclass
class RingCosts:
    """Measured costs (ms).  ``core[(frames, g)]`` / ``dense[(frames, g)]``:
    one job over g chunks of ``frames`` frames; ``t_align``: one alignment
    beside a gated encode, ``t_align_alone``: with the rank's encodes done;
    ``t_pause``: encode time one alignment costs its rank (the gate's pause);
    ``t_align_ungated`` / ``t_pause_ungated``: the same without the gate (the
    alignment shares the CUs with the encode: slower, but it costs the encode
    less); ``hop``: one baton send/recv between ranks; ``gather``: the end-of-sequence
    all-gather + depth scaling."""
    core: Dict[Tuple[int, int], float]
    dense: Dict[Tuple[int, int], float]
    t_align: float
    t_align_alone: float
    t_pause: float
    t_align_ungated: float = 7.7
    t_pause_ungated: float = 1.6
    hop: float = 0.25
    gather: float = 0.5
    ship: float = 0.3
    source: str = ""

    def job_ms(self, kind: str, frames: int, g: int) -> float:
        if kind == "enc":
            return self.job_ms("core", frames, g) + self.job_ms("dense", frames, g)
        tab = self.core if kind == "core" else self.dense
        if (frames, g) in tab:
            return tab[(frames, g)]
        # nearest measured entry, scaled by the work ratio (frames x group size)
        fr, gg = min(tab, key=lambda k: (abs(k[0] - frames), abs(k[1] - g)))
        return tab[(fr, gg)] * (frames * g) / (fr * gg)

    def to_json(self) -> dict:
        d = asdict(self)
        d["core"] = {f"{k[0]}x{k[1]}": v for k, v in self.core.items()}
        d["dense"] = {f"{k[0]}x{k[1]}": v for k, v in self.dense.items()}
        return d

    @staticmethod
    def from_json(d: dict) -> "RingCosts":
        d = dict(d)
        for key in ("core", "dense"):
            d[key] = {tuple(int(x) for x in k.split("x")): float(v) for k, v in d[key].items()}
        return RingCosts(**d)


# Default costs: 16-frame 154x518 chunks (BASELINE configs[3] / [4]) on one MI355X,
# measured by bench.py --config 3 (`ring_model.costs`, profiles/r9); only the RELATIVE
# costs steer the plan.  Other shapes scale by frames x group size (job_ms).
DEFAULT_COSTS = RingCosts(
    core={(16, 1): 25.0, (16, 2): 47.2, (16, 3): 61.5, (8, 1): 18.0},
    dense={(16, 1): 7.2, (16, 2): 12.5, (16, 3): 17.8, (8, 1): 5.0},
    t_align=2.58, t_align_alone=2.34, t_pause=3.57, t_align_ungated=6.85, t_pause_ungated=1.39, hop=0.105, ship=0.29,
    gather=0.5,
    source="bench.py --config 3, round 5 (profiles/r10/c3.json: CP-side gate wait, in-workgroup split linears)")


def load_costs() -> RingCosts:
    """VGGT_RING_COSTS=<json file> (a bench line's ``ring_model.costs``) or the defaults."""
    p = os.environ.get("VGGT_RING_COSTS")
    if p:
        with open(p) as fh:
            d = json.load(fh)
        return RingCosts.from_json(d.get("ring_model", {}).get("costs", d))
    return DEFAULT_COSTS


# ------------------------------------------------------------------ plans
def compositions(n: int, cap: int) -> List[Tuple[int, ...]]:
    """All ordered ways to write n as a sum of parts in 1..cap."""
    if n == 0:
        return [()]
    out = []
    for first in range(1, min(cap, n) + 1):
        out.extend((first,) + rest for rest in compositions(n - first, cap))
    return out


def candidate_sizes(n: int, cap: int, full_upto: int = 8) -> List[Tuple[int, ...]]:
    """Group-size sequences tried for a run of n chunks: every composition
    for short runs (a W >= 4 rank owns <= 11 of 43 chunks); for long runs
    (W = 1, 2) a head of up to 2 chunks in any composition, a uniform middle
    of groups of g, and a tail of up to 2 chunks in any composition."""
    if n <= full_upto:
        return compositions(n, cap)
    out = set()
    ends = [c for k in range(0, 3) for c in compositions(k, cap)]
    for head in ends:
        for tail in ends:
            mid = n - sum(head) - sum(tail)
            if mid < 0:
                continue
            for g in range(1, cap + 1):
                body = (g,) * (mid // g) + ((mid % g,) if mid % g else ())
                out.add(tuple(head) + body + tuple(tail))
    return sorted(out)


def runs_of(own: Sequence[int], lengths: Sequence[int]) -> List[List[int]]:
    """Maximal runs of consecutive own chunks with equal length (only those can share an encode)."""
    out: List[List[int]] = []
    for i in own:
        if out and lengths[out[-1][-1]] == lengths[i]:
            out[-1].append(i)
        else:
            out.append([i])
    return out


def make_jobs(groups: Sequence[Sequence[int]], policy: str) -> List[Job]:
    """Job list of one rank.  policy: "with" (DPT inside each encode), "lag"
    (each group's DPT after the NEXT group's core), "end" (every core first)."""
    gs = [tuple(g) for g in groups]
    if policy == "with":
        return [("enc", g) for g in gs]
    if policy == "end":
        return [("core", g) for g in gs] + [("dense", g) for g in gs]
    if policy == "lag":
        jobs: List[Job] = []
        for k, g in enumerate(gs):
            jobs.append(("core", g))
            if k > 0:
                jobs.append(("dense", gs[k - 1]))
        if gs:
            jobs.append(("dense", gs[-1]))
        return jobs
    raise ValueError(policy)


def held_peak(jobs: Sequence[Job]) -> int:
    """Most chunks whose core results wait on the device for their DPT job at
    any point of one rank's job list ("end" holds every core until the last
    encode; "lag" at most two groups; "with" none)."""
    held = peak = 0
    for kind, g in jobs:
        if kind == "core":
            held += len(g)
            peak = max(peak, held)
        elif kind == "dense":
            held -= len(g)
    return peak


def split_groups(own: Sequence[int], lengths: Sequence[int], sizes: Sequence[int]) -> List[List[int]]:
    """Cut the rank's longest equal-length run by ``sizes``; other runs (a
    tail chunk of another length) become groups of their own."""
    runs = runs_of(own, lengths)
    main = max(range(len(runs)), key=lambda k: len(runs[k])) if runs else -1
    out: List[List[int]] = []
    for k, run in enumerate(runs):
        if k != main:
            out.append(list(run))
            continue
        o = 0
        for s in sizes:
            out.append(list(run[o:o + s]))
            o += s
    return out


@dataclass
class RankPlan:
    jobs: List[Job]
    sizes: Tuple[int, ...] = ()
    policy: str = "with"
    gated: bool = True
    # align_rank[i]: the rank that runs chunk i's alignment (the same tuple in every
    # rank's plan); () = the owner (i mod W).  An alignment away from its owner gets
    # the chunk's core outputs by one point-to-point "ship" (the alignment head's
    # prefix rows + the camera pose encoding, ~27 MB at 154x518)
    align_rank: Tuple[int, ...] = ()


@dataclass
class Prediction:
    total_ms: float
    align_start: List[float] = field(default_factory=list)
    align_end: List[float] = field(default_factory=list)
    rank_finish: List[float] = field(default_factory=list)


def _timeline(jobs: Sequence[Job], lengths, costs: RingCosts, pauses: Sequence[float],
              t_pause: float) -> List[float]:
    """End time of every job on one encode stream (jobs back to back from 0);
    each alignment starting at p while a job runs pauses that job t_pause."""
    t = 0.0
    ends = []
    ps = sorted(pauses)
    for kind, g in jobs:
        dur = costs.job_ms(kind, lengths[g[0]], len(g))
        start = t
        end = start + dur
        lo = bisect.bisect_left(ps, start)
        while True:
            k = bisect.bisect_left(ps, end) - lo
            new = start + dur + k * t_pause
            if new == end:
                break
            end = new
        ends.append(end)
        t = end
    return ends


def simulate(lengths: Sequence[int], W: int, plans: Sequence[RankPlan], costs: RingCosts) -> Prediction:
    """Predicted sequence time of the ring: chunk i's core encode on its owner
    (i mod W), its alignment on plans[*].align_rank[i] (default the owner)."""
    n = len(lengths)
    core_job: Dict[int, Tuple[int, int]] = {}
    for r, pl in enumerate(plans):
        for j, (kind, g) in enumerate(pl.jobs):
            if kind in ("enc", "core"):
                for i in g:
                    core_job[i] = (r, j)
    ar = plans[0].align_rank if plans and plans[0].align_rank else tuple(i % W for i in range(n))
    pauses: List[List[float]] = [[] for _ in range(W)]
    a_s: List[float] = []
    a_e: List[float] = []
    tp = [costs.t_pause if pl.gated else costs.t_pause_ungated for pl in plans]
    for i in range(n):
        r, j = core_job[i]
        a = ar[i]
        s = _timeline(plans[r].jobs, lengths, costs, pauses[r], tp[r])[j]
        if a != r:
            s += costs.ship
        if i > 0:
            s = max(s, a_e[-1] + (costs.hop if ar[i - 1] != a else 0.0))
        tla = _timeline(plans[a].jobs, lengths, costs, pauses[a], tp[a])
        busy = bool(tla) and s < tla[-1]  # the aligning rank still has encode work queued at s
        if busy:
            pauses[a].append(s)
        a_s.append(s)
        a_e.append(s + ((costs.t_align if plans[a].gated else costs.t_align_ungated) if busy
                        else costs.t_align_alone))
    fin = [(_timeline(pl.jobs, lengths, costs, pauses[r], tp[r]) or [0.0])[-1] for r, pl in enumerate(plans)]
    total = max(max(fin), a_e[-1] if a_e else 0.0) + costs.gather
    return Prediction(total, a_s, a_e, fin)


_POLICIES = ("with", "lag", "end")


def plan_ring(lengths: Sequence[int], W: int, costs: Optional[RingCosts] = None, cap: int = 3,
              policies: Sequence[str] = _POLICIES, gates: Sequence[bool] = (True, False),
              sweeps: int = 2, offload: bool = True, refine: bool = True,
              max_held: Optional[int] = None) -> Tuple[List[RankPlan], Prediction]:
    """Per-rank plans minimising the predicted sequence time: each rank's
    longest equal-length run is cut into groups of <= cap chunks (every
    composition tried) under each DPT placement policy, gated or not, rank by rank, a few
    coordinate-descent sweeps from the best uniform choice.  ``max_held``
    bounds device memory: no rank's plan may hold more than that many chunks'
    core results waiting for their DPT job (``held_peak``; the caller derives
    it from a byte budget), so a long sequence falls back from "end" to "lag"
    or "with" instead of growing without bound.  Then (offload)
    alignments move, one at a time, from the rank that finishes last to the
    ranks that finish first while the prediction improves: 43 chunks over 8
    ranks leave two ranks six chunks, and their alignments' gate pauses are
    what keeps them last.  With ``refine``, one more pass over each rank's
    options with the alignments fixed where they went, then the moves again.
    Deterministic, so every rank computes the same plans."""
    costs = costs or load_costs()
    n = len(lengths)
    owns = [list(range(r, n, W)) for r in range(W)]
    options: List[List[Tuple[Tuple[int, ...], str, bool]]] = []
    for r in range(W):
        runs = runs_of(owns[r], lengths)
        m = max((len(x) for x in runs), default=0)
        opts = [(c, p, gt) for c in candidate_sizes(m, cap) for p in policies for gt in gates]
        if max_held is not None:
            fits = [o for o in opts
                    if held_peak(make_jobs(split_groups(owns[r], lengths, o[0]), o[1])) <= max_held]
            # "with" holds nothing, so it always fits
            opts = fits or [(c, "with", gt) for c in candidate_sizes(m, cap) for gt in gates]
        options.append(opts)

    def build(choice):
        return [RankPlan(make_jobs(split_groups(owns[r], lengths, c), p), c, p, gt)
                for r, (c, p, gt) in enumerate(choice)]

    def score(choice):
        pr = simulate(lengths, W, build(choice), costs)
        return (round(pr.total_ms, 6), round(sum(pr.rank_finish), 6)), pr

    # starts: for each DPT policy, the best choice applied to every rank alike (by the
    # pattern of the largest rank); each start is refined by coordinate descent
    uniform = {}
    for c, p, gt in options[0]:
        choice = []
        for r in range(W):
            m = sum(c)
            mine = max((len(x) for x in runs_of(owns[r], lengths)), default=0)
            cc = c if mine == m else _fit(c, mine, cap)
            if max_held is not None and held_peak(make_jobs(split_groups(owns[r], lengths, cc), p)) > max_held:
                p_r = "with"  # the fitted composition of a longer run may hold one chunk more
            else:
                p_r = p
            choice.append((cc, p_r, gt))
        sc, pr = score(choice)
        if p not in uniform or sc < uniform[p][0]:
            uniform[p] = (sc, choice, pr)
    best = None
    for p in sorted(uniform):
        sc, choice, pr = uniform[p]
        for _ in range(sweeps):
            changed = False
            for r in range(W):
                for opt in options[r]:
                    if opt == choice[r]:
                        continue
                    trial = list(choice)
                    trial[r] = opt
                    s2, p2 = score(trial)
                    if s2 < sc:
                        sc, choice, pr, changed = s2, trial, p2, True
            if not changed:
                break
        if best is None or sc < best[0]:
            best = (sc, choice, pr)
    sc, choice, pr = best
    plans = build(choice)
    if offload and W > 1:
        plans, pr = _offload(lengths, W, plans, costs, pr)
    if offload and W > 1 and refine:
        # one more pass over each rank's plan with the alignments where the moves put
        # them (a rank relieved of its alignments may now prefer other groups), then
        # the moves again from there
        key = lambda p: (round(p.total_ms, 6), round(max(p.rank_finish), 6), round(sum(p.rank_finish), 6))  # noqa: E731
        ar = list(plans[0].align_rank)
        changed = False
        for r in range(W):
            for opt in options[r]:
                if opt == choice[r]:
                    continue
                trial = list(choice)
                trial[r] = opt
                tp = build(trial)
                for pl in tp:
                    pl.align_rank = tuple(ar)
                p2 = simulate(lengths, W, tp, costs)
                if key(p2) < key(pr):
                    choice, plans, pr, changed = trial, tp, p2, True
        if changed:
            plans, pr = _offload(lengths, W, plans, costs, pr, ar)
    return plans, pr


def _offload(lengths, W, plans, costs, pr, ar0=None):
    """Greedy alignment moves off the last-finishing rank (see plan_ring), from
    the owners (or from ``ar0``)."""
    n = len(lengths)
    ar = list(ar0) if ar0 is not None else list(i % W for i in range(n))

    def with_ar(a):
        for pl in plans:
            pl.align_rank = tuple(a)
        return simulate(lengths, W, plans, costs)

    best = with_ar(ar)
    key = lambda p: (round(p.total_ms, 6), round(max(p.rank_finish), 6), round(sum(p.rank_finish), 6))  # noqa: E731
    for _ in range(n):
        R = max(range(W), key=lambda r: best.rank_finish[r])
        targets = sorted(range(W), key=lambda r: best.rank_finish[r])[:3]
        cand = None
        # the last-finishing rank's alignments, and the chain's tail (alignments that start
        # after the first rank has run out of encode work run there at their alone speed)
        idle_from = min(best.rank_finish)
        movable = [i for i in range(n) if ar[i] == R or best.align_start[i] >= idle_from]
        for i in movable:
            for q in targets:
                if q == R:
                    continue
                trial = list(ar)
                trial[i] = q
                p2 = with_ar(trial)
                if key(p2) < key(best) and (cand is None or key(p2) < key(cand[1])):
                    cand = (trial, p2)
        if cand is None:
            break
        ar, best = cand
    with_ar(ar)
    return plans, best


def _fit(c: Tuple[int, ...], m: int, cap: int) -> Tuple[int, ...]:
    """Adapt a composition to a run of m chunks: trim from the front or extend with 1s at the front."""
    c = list(c)
    while sum(c) > m:
        c[0] -= 1
        if c[0] == 0:
            c.pop(0)
    while sum(c) < m:
        c.insert(0, 1)
    return tuple(c)


def legacy_plans(lengths: Sequence[int], W: int, cap: int = 3) -> List[RankPlan]:
    """Round-4 schedule for comparison: each rank's own consecutive equal-length
    chunks greedily in groups of ``cap``, DPT inside each encode."""
    n = len(lengths)
    plans = []
    for r in range(W):
        groups: List[List[int]] = []
        for i in range(r, n, W):
            if groups and len(groups[-1]) < cap and lengths[groups[-1][-1]] == lengths[i]:
                groups[-1].append(i)
            else:
                groups.append([i])
        plans.append(RankPlan(make_jobs(groups, "with"), tuple(len(g) for g in groups), "with"))
    return plans


def enqueue_order(plan: RankPlan, own: Sequence[int], rank: Optional[int] = None
                  ) -> List[Tuple[str, Tuple[int, ...]]]:
    """The host-side order in which the ring issues this rank's work: its jobs
    in plan order; after a job, the "ship" of each chunk in it whose alignment
    runs on another rank; and alignment i right after the job FOLLOWING the
    last job that produced a core of one of this rank's chunks <= i (one job of
    look-ahead keeps the encode stream fed while the host waits on a
    host-blocking baton; over RCCL nothing blocks).  Every own chunk < i is
    thus encoded and shipped before alignment i is issued, so a host-blocking
    baton can never wait on this rank's own later work.  Returns ("job", (j,)),
    ("ship", (i,)) and ("align", (i,)) entries."""
    jobs = plan.jobs
    ar = plan.align_rank
    core_at = {}
    for j, (kind, g) in enumerate(jobs):
        if kind in ("enc", "core"):
            for i in g:
                core_at[i] = j
    aligns = list(own) if not ar else [i for i in range(len(ar)) if ar[i] == rank]
    own_sorted = sorted(own)
    out: List[Tuple[str, Tuple[int, ...]]] = []
    issued = -1

    def issue_to(need):
        nonlocal issued
        while issued < need:
            issued += 1
            out.append(("job", issued))
            kind, g = jobs[issued]
            if ar and kind in ("enc", "core"):
                out.extend(("ship", (c,)) for c in g if ar[c] != rank)

    for i in aligns:
        prior = [core_at[c] for c in own_sorted if c <= i]
        if prior:
            issue_to(min(max(prior) + 1, len(jobs) - 1))
        out.append(("align", (i,)))
    issue_to(len(jobs) - 1)
    return out


def predict_scaling(lengths: Sequence[int], costs: RingCosts, worlds=(1, 2, 4, 8), offload: bool = False) -> dict:
    """Predicted sequence time at each W with the plans the pipeline runs by
    default (``offload``: alignments moved off their owner, VGGT_RING_OFFLOAD),
    the other offload setting beside it, and the round-4 schedule's."""
    out = {}
    for W in worlds:
        plans, pr = plan_ring(lengths, W, costs, offload=offload)
        _, pr_alt = plan_ring(lengths, W, costs, offload=not offload) if W > 1 else (None, pr)
        leg = simulate(lengths, W, legacy_plans(lengths, W), costs)
        moved = [i for i, a in enumerate(plans[0].align_rank) if a != i % W] if plans[0].align_rank else []
        out[str(W)] = {"T_ms": round(pr.total_ms, 1),
                       ("T_ms_with_offload" if not offload else "T_ms_no_offload"): round(pr_alt.total_ms, 1),
                       "T_ms_round4_schedule": round(leg.total_ms, 1), "alignments_moved": moved,
                       "plans": [{"groups": [list(g) for k, g in pl.jobs if k in ("enc", "core")],
                                  "policy": pl.policy, "gated": pl.gated} for pl in plans[:min(W, 3)]]}
    return out
