"""dkg_amd — MI355X-native (gfx950 HIP) backend for the share-generation / share-verification hot
path of the danielSanchezQ/dkg Pedersen-VSS DKG over Ristretto255.  See DESIGN.md."""
from ._lib import ACCEPT, MISSING, REJECT, SELF, SKIPPED, DkgError, lib  # noqa: F401
from .api import (Backend, BatchResult, MultiBackend, CeremonyResult, Environment, ceremony_batch_device,  # noqa: F401
                  ceremony_batch_verify, dealer_coefficients, enc_randomness, env_check, packed_row_words, shard_range,
                  shard_rows, split_multipliers)

__all__ = ["Backend", "MultiBackend", "Environment", "CeremonyResult", "BatchResult", "DkgError", "dealer_coefficients", "env_check",
           "ceremony_batch_device", "ceremony_batch_verify", "enc_randomness", "split_multipliers", "lib",
           "shard_range", "shard_rows", "packed_row_words",
           "ACCEPT", "REJECT", "SELF", "SKIPPED", "MISSING"]
