"""CMA-ES eigensolver schedule from measured convergence (round 6; CMAES._poll_eig_health).

Host logic only: the solve reports of a run are fed through the pinned-ring protocol with
synthetic rows, and the schedule must (1) start cold, (2) move down one level after
DOWN_STREAK consecutive solves that fit the next shorter schedule with a slot to spare,
(3) go back up at the first capped / slow solve — relative to the level that solve ran at, so
the solves still in flight at the short level do not over-escalate — and (4) restart cold in a
new run (the escalation state lived across wf.init)."""
import torch

from evoxmi import config
from evoxmi.algorithms import CMAES


class _Done:
    def synchronize(self):
        pass


def _algo(d=1000):
    a = CMAES(center_init=torch.zeros(d), init_stdev=1.0, pop_size=10000)
    a.setup(torch.zeros(2, dtype=torch.int64))
    a._eig_ring = torch.full((CMAES.ESC_RING, 5), -1.0, dtype=torch.float64)
    return a


def _run(a, solves):
    """Drive one step per (iterations, capped) pair; returns the variant of every step."""
    out = []
    sc = a._sched()
    for k, (iters, capped) in enumerate(solves):
        a._poll_eig_health(sc)
        sc["last"] = sc["level"]
        out.append(sc["level"])
        # the step's solve reports into ring slot k, then the step's "event" is recorded
        a._eig_ring[k % CMAES.ESC_RING] = torch.tensor([1e-6, 1.0 if capped else 0.0, float(iters), 0.0, float(k)],
                                                       dtype=torch.float64)
        sc["pending"].append((k, _Done(), sc["last"]))
        sc["enqueued"] = k + 1
    return out


def test_schedule_starts_cold_and_moves_down_on_measured_convergence():
    a = _algo()
    cold, warm, warm6, late = (a._level_slots(l) for l in (3, 2, 1, 0))
    assert (late, warm6, warm, cold) == (config.get("sbr_late_iters"), config.get("sbr_device_iters") - 1, config.get("sbr_device_iters"),
                                         config.get("sbr_cold_iters"))
    # cold-start solves need 10-12 iterations, then 5-6 (fit warm), then 4 (fit late)
    solves = [(12, False), (10, False), (6, False), (6, False), (6, False), (5, False), (5, False)] + [(4, False)] * 10
    lv = _run(a, solves)
    assert lv[0] == 3 and lv[1] == 3
    first_warm = lv.index(2)
    # two consecutive cold solves with ≤ warm − 1 iterations, read two steps late
    assert first_warm == 2 + 2 + 1
    first_late = lv.index(0)
    assert first_late > first_warm and all(v == 0 for v in lv[first_late:])
    assert 1 in lv[first_warm:first_late]  # through the one-slot-shorter warm schedule
    assert a.schedule_escalations == 0


def test_capped_late_solve_escalates_once_and_slow_solve_returns_to_warm():
    a = _algo()
    sc = a._sched()
    sc["level"] = 0  # settled
    solves = [(4, False)] * 3 + [(5, True)] * 2 + [(5, False)] * 7
    lv = _run(a, solves)
    # solve 3 capped at the late level → warm from step 3 + ESC_LAG on; the two capped solves
    # still in flight at the late level do not push it to cold
    assert lv[:5] == [0, 0, 0, 0, 0]
    assert lv[5] == 1 and max(lv) == 1  # one level up: the shorter warm schedule
    assert a.schedule_escalations == 2
    # a solve that converged only in the late schedule's last slot also moves the run up
    b = _algo()
    b._sched()["level"] = 0
    lv = _run(b, [(4, False)] * 2 + [(config.get("sbr_late_iters"), False)] + [(5, False)] * 5)
    assert 1 in lv and b.schedule_escalations == 0


def test_new_run_restarts_the_schedule():
    a = _algo()
    _run(a, [(4, False)] * 3)
    a._sched()["level"] = 0
    a.setup(torch.zeros(2, dtype=torch.int64))
    sc = a._sched()
    assert sc["level"] == CMAES.TOP and sc["enqueued"] == 0 and not sc["pending"] and a.schedule_escalations == 0
