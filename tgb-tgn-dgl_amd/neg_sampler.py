"""Drop-in for the reference's neg_sampler.py (NegLinkSamplerDest) — device counter-based sampler."""
from tgnx.neg import NegLinkSamplerDest  # noqa: F401
