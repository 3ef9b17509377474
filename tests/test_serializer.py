"""Viewer JSON (reference serializer.py:20-49, read by landmark_map/utils/deserializer.py):
the vectorised particle block is byte-identical to json.dump(..., indent=4)."""
import json

import numpy as np

from fast_slam_2 import DirectedPoint, EvaluationResults, Point, Serializer


class _FakeFilter:
    def __init__(self, x, y, yaw):
        self._p = (x, y, yaw)

    def poses(self):
        return self._p


class _View(list):
    pass


def _args(n, rng):
    x = rng.normal(0, 10, n)
    y = rng.normal(0, 1e-3, n)
    yaw = rng.uniform(-np.pi, np.pi, n)
    x[:5] = [0.0, -0.0, 1.0, 1e300, 5e-324]
    y[:4] = [np.nan, np.inf, -np.inf, 2.0]
    est, act = DirectedPoint(0.1, 0.2, 0.3), DirectedPoint(1.0, 2.0, -0.5)
    lms = [Point(float(a), float(b)) for a, b in rng.normal(0, 5, (7, 2))]
    res = EvaluationResults("2024-01-01 00:00:00", 0.1, 0.2, 0.3, 0.4, 0.5)
    return x, y, yaw, est, act, lms, res


def test_particle_block_matches_json_dump():
    rng = np.random.default_rng(3)
    for n in (0, 1, 257):
        x, y, yaw, est, act, lms, res = _args(n, rng) if n >= 5 else (
            rng.normal(size=n), rng.normal(size=n), rng.normal(size=n), *_args(8, rng)[3:])
        plain = [DirectedPoint(float(a), float(b), float(c)) for a, b, c in zip(x, y, yaw)]
        want = json.dumps({"estimated_robot_pos": est.to_dict(), "actual_robot_pos": act.to_dict(),
                           "particles": [p.to_dict() for p in plain],
                           "landmarks": [lm.to_dict() for lm in lms], "results": res.to_dict()}, indent=4)
        view = _View()
        view._filter = _FakeFilter(x, y, yaw)
        assert Serializer.to_json(est, act, view, lms, res) == want
        assert Serializer.to_json(est, act, plain, lms, res) == want


def test_schema_round_trip():
    rng = np.random.default_rng(4)
    x, y, yaw, est, act, lms, res = _args(20, rng)
    view = _View()
    view._filter = _FakeFilter(x, y, yaw)
    d = json.loads(Serializer.to_json(est, act, view, lms, res))
    assert set(d) == {"estimated_robot_pos", "actual_robot_pos", "particles", "landmarks", "results"}
    assert len(d["particles"]) == 20 and set(d["particles"][7]) == {"x", "y", "yaw"}
    assert d["particles"][7]["yaw"] == yaw[7]
    assert set(d["landmarks"][0]) == {"x", "y"}
