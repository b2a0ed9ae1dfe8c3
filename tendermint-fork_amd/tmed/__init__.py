"""tmed — MI355X-native batch ed25519 verification for Tendermint commit verification.

Host-side mirror of the reference interfaces on the hot path
(``crypto/ed25519`` PubKey.VerifySignature, ``types.ValidatorSet.VerifyCommit*``)
over the gfx950 C ABI in ``include/tmed25519.h``.
"""
from ._native import LIB_PATH, TmedError, lib  # noqa: F401
from .engine import Engine, PinnedBuffer, pack_messages  # noqa: F401
