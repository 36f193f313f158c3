"""MI355X-native batch engine for SafeStake's threshold-BLS hot path (BLS12-381).

The compute path is libssbls.so (hand-written HIP for gfx950, C ABI in include/ssbls.h);
this package is the host-side mirror of the reference's threshold-signature API.
"""
from .threshold import (  # noqa: F401
    DST, INFINITY_SIGNATURE, DvfError, DifferentLength, InsufficientSignatures, InvalidOperatorId,
    InsufficientValidSignatures, BadSignatureEncoding, Engine, ThresholdJob, ThresholdSignature,
)
from .collector import SlotCollector  # noqa: F401,E402
