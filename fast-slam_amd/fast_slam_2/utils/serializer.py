"""JSON wire format of the viewer (reference: fast_slam_2/utils/serializer.py:20-49,
read back by landmark_map/utils/deserializer.py).

Same file, same schema, same text as the reference's `json.dump(..., indent=4)`.
Given FastSLAM2.particles, the particle poses come from one structure-of-arrays
download (x, y, yaw) and the particle block is written by a vectorised emitter
that produces exactly the text json's encoder would, so a 1e6-particle snapshot
does not build 1e6 Python objects.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np

_IND = "    "


def _num(v: float) -> str:
    """json.dumps of a float (float.__repr__, NaN / Infinity spellings)."""
    if v != v:
        return "NaN"
    if math.isinf(v):
        return "Infinity" if v > 0 else "-Infinity"
    return float.__repr__(float(v))


def _poses_block(x, y, yaw, depth: int) -> str:
    """Text of a JSON list of {"x", "y", "yaw"} objects at nesting depth `depth`."""
    if len(x) == 0:
        return "[]"
    i1, i2 = _IND * (depth + 1), _IND * (depth + 2)
    head = i1 + "{\n" + i2 + '"x": '
    mid1 = ",\n" + i2 + '"y": '
    mid2 = ",\n" + i2 + '"yaw": '
    tail = "\n" + i1 + "}"
    items = [head + a + mid1 + b + mid2 + c + tail
             for a, b, c in zip(map(_num, x.tolist()), map(_num, y.tolist()), map(_num, yaw.tolist()))]
    return "[\n" + ",\n".join(items) + "\n" + _IND * depth + "]"


class Serializer:
    shared_path = "workspace/shared"
    file_name = "fast_slam.json"
    file_path = os.path.join(shared_path, file_name)

    @staticmethod
    def to_json(estimated_robot_pos, actual_robot_pos, particles, landmarks, results) -> str:
        fs = getattr(particles, "_filter", None)
        if fs is None:
            return json.dumps({
                "estimated_robot_pos": estimated_robot_pos.to_dict(),
                "actual_robot_pos": actual_robot_pos.to_dict(),
                "particles": [p.to_dict() for p in particles],
                "landmarks": [lm.to_dict() for lm in landmarks],
                "results": results.to_dict(),
            }, indent=4)
        x, y, yaw = fs.poses()
        marker = "\x00particles\x00"
        text = json.dumps({
            "estimated_robot_pos": estimated_robot_pos.to_dict(),
            "actual_robot_pos": actual_robot_pos.to_dict(),
            "particles": marker,
            "landmarks": [lm.to_dict() for lm in landmarks],
            "results": results.to_dict(),
        }, indent=4)
        return text.replace(json.dumps(marker), _poses_block(x, y, yaw, 1), 1)

    @staticmethod
    def serialize(estimated_robot_pos, actual_robot_pos, particles, landmarks, results):
        """Write the snapshot to workspace/shared/fast_slam.json (serializer.py:20-49)."""
        text = Serializer.to_json(estimated_robot_pos, actual_robot_pos, particles, landmarks, results)
        os.makedirs(Serializer.shared_path, exist_ok=True)
        with open(Serializer.file_path, "w") as f:
            f.write(text)
