"""Host-side pose metrics of ``/root/reference/pose_evaluation.py`` (numpy, [frames, joints, 3] in mm).

The reference's evaluation runs on the host after the forward (train_hier_networks.py:323,
train_dense_networks.py:208, train_dense_hier_networks.py:324 call ``getMeanError_np``); these are
the same NaN-aware reductions, checked against the reference's own functions executed on the same
inputs (tests/golden/make_crop_fixtures.py, tests/test_crop_reference.py).
"""
from __future__ import annotations

import numpy as np


def _joint_dist(labels, results, axis=2):
    d = np.asarray(labels) - np.asarray(results)
    return np.sqrt(np.square(d).sum(axis=axis))


def getMeanError_np(labels, results):
    """Mean over frames of the mean joint distance (pose_evaluation.py:10-15)."""
    return np.nanmean(np.nanmean(_joint_dist(labels, results), axis=1))


def getMaxError_np(labels, results):
    """Largest joint distance (pose_evaluation.py:18-24)."""
    return np.nanmax(_joint_dist(labels, results))


def getMean_np(labels, results):
    """Mean joint distance per joint over a [frames, 3] pair (pose_evaluation.py:26-28)."""
    return np.nanmean(_joint_dist(labels, results, axis=1), axis=0)


def getNumFramesWithinMaxDist(labels, results, dist):
    """Frames whose worst joint is within ``dist`` mm (pose_evaluation.py:63-69)."""
    return (np.nanmax(_joint_dist(labels, results), axis=1) <= dist).sum()


def getNumFramesWithinMeanDist(labels, results, dist):
    """Frames whose mean joint distance is within ``dist`` mm (pose_evaluation.py:72-78)."""
    return (np.nanmean(_joint_dist(labels, results), axis=1) <= dist).sum()


def getJointMeanError(labels, results, jointID):
    """Mean distance of one joint over the frames (pose_evaluation.py:81-88)."""
    lab, res = np.asarray(labels), np.asarray(results)
    return np.nanmean(np.sqrt(np.square(lab[:, jointID, :] - res[:, jointID, :]).sum(axis=1)))
