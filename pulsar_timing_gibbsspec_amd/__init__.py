"""MI355X-native free-spectrum Gibbs sampler for pulsar-timing arrays.

Drop-in for the hot path of astrolamb/pulsar_timing_gibbsspec: the
``PulsarBlockGibbs`` / ``PTABlockGibbs`` surface over hand-written gfx950 HIP
kernels reached through the C-ABI in ``include/pulsar_gibbs.h``.
"""
__version__ = "0.1.0"

from .pulsar_gibbs import PulsarBlockGibbs  # noqa: F401,E402
from .pta_gibbs import PTABlockGibbs  # noqa: F401,E402
