"""Caller-side engine around the DSTDGCN hot path.

Mirrors the reference's ``engine/`` package: ``PredictionEngine`` /
``ModelWrapper`` (engine/prediction.py), ``mpjpe_error_3d`` / ``AccumLoss``
(engine/utils/loss.py) and the ``tsc`` transforms (engine/utils/transform.py).
Loss, loss gradient and the test metric run as HIP kernels
(include/dstd_gcn_train.h); training steps and test batches never call
``.item()`` -- each epoch / test run synchronises once at its end.
"""
from .loss import AccumLoss, DeviceAccum, mpjpe_error_3d  # noqa: F401
from .prediction import ModelWrapper, PredictionEngine  # noqa: F401
from .transform import tsc_inverse, tsc_transform  # noqa: F401
