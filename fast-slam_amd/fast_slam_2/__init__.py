"""fast_slam_2 -- MI355X-native drop-in for the reference's FastSLAM 2.0 hot path.

Same public names as cy-rae/fast-slam's `fast_slam_2` package
(fast_slam_2/__init__.py:5-22).  The particle update, ICP, LineFilter and the
association / Mahalanobis helpers and the known-landmark clustering
(update_known_landmarks / cluster_points) run in libfs2.so (HIP, gfx950);
Serializer writes the viewer's JSON from one device download; the landmark
front-end (LandmarkUtils.get_measurements_to_landmarks, HoughTransformation)
runs batched on the device too.  Robot keeps its ICP odometry
(get_transformation_icp); its laser / motor calls and EvaluationUtils are
simulator-bound (HAL) and outside this build's scope.
"""
from .algorithms.fast_slam_2 import FastSLAM2
from .algorithms.hough_transformation import HoughTransformation
from .algorithms.icp import ICP
from .algorithms.line_filter import LineFilter
from .models.directed_point import DirectedPoint
from .models.evaluation_results import EvaluationResults
from .models.landmark import Landmark
from .models.measurement import Measurement
from .models.particle import Particle
from .models.point import Point
from .models.robot import Robot
from .utils.geometry_utils import GeometryUtils
from .utils.landmark_utils import LandmarkUtils
from .utils.serializer import Serializer

_OUT_OF_SCOPE = {"EvaluationUtils"}


def release_cached_memory() -> int:
    """Release the device memory libfs2 keeps from closed handles for later pool
    growth (kept only when FS2_VMM_CACHE_MB opts in; fs2.h
    fs2_release_cached_memory).  Returns the bytes released."""
    from . import _native
    return int(_native.load().fs2_release_cached_memory())


def __getattr__(name):
    if name in _OUT_OF_SCOPE:
        raise ImportError(f"fast_slam_2.{name} drives the JdeRobot simulator (HAL), which this "
                          f"build does not replace (SURVEY.md §2)")
    raise AttributeError(name)


__all__ = ["FastSLAM2", "HoughTransformation", "ICP", "LineFilter", "DirectedPoint", "EvaluationResults", "Landmark",
           "Measurement", "Particle", "Point", "Robot", "GeometryUtils", "LandmarkUtils", "Serializer",
           "release_cached_memory"]
