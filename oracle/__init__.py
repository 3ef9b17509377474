"""CPU oracle for the FastSLAM 2.0 hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product path (fast-slam_amd/, libfs2.so) never
imports, links or calls it.
"""
