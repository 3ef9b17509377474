"""Configuration knobs of the FastSLAM 2.0 engine (names and defaults of the
reference's fast_slam_2/config.py:7-21).

Unlike the reference, which binds these by name at import time in every module
(SURVEY.md Q15), FastSLAM2() reads them from this module when it is
constructed, so assigning `fast_slam_2.config.NUM_PARTICLES = ...` before
construction takes effect.
"""
import numpy as np

NUM_PARTICLES = 20
TRANSLATION_NOISE = 0.0055
ROTATION_NOISE = 0.001
MEASUREMENT_NOISE = np.array([[0.001, 0.0], [0.0, 0.001]])
MAXIMUM_LANDMARK_DISTANCE = 8
# Kept for API compatibility: the reference's per-phase thread pool
# (fast_slam_2.py:42-53).  The device runs every particle in parallel.
NUM_THREAD = 20

# Not a reference knob.  The landmark front-end (LandmarkUtils.get_measurements_to_landmarks)
# follows numpy's scalar promotion rules: False = numpy >= 2 (NEP 50: intersections,
# cluster centres and corners stay float32; what this repository's fixtures pin),
# True = numpy 1.x (the reference's requirements.txt pins numpy~=1.24: float64 from
# the back-conversion to metres on).  The two differ at float32 rounding (~1e-7).
FRONTEND_NUMPY1_PROMOTION = False
