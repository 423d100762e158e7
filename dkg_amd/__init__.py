"""dkg_amd — MI355X-native (gfx950 HIP) backend for the share-generation / share-verification hot
path of the danielSanchezQ/dkg Pedersen-VSS DKG over Ristretto255.  See DESIGN.md."""
from ._lib import ACCEPT, REJECT, SELF, SKIPPED, DkgError, lib  # noqa: F401
from .api import Backend, CeremonyResult, Environment, dealer_coefficients, env_check  # noqa: F401

__all__ = ["Backend", "Environment", "CeremonyResult", "DkgError", "dealer_coefficients", "env_check", "lib",
           "ACCEPT", "REJECT", "SELF", "SKIPPED"]
