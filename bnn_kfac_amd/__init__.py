"""bnn_kfac_amd — MI355X-native KFAC curvature engine (drop-in for the KFAC hot path
of TianmingQiu/BNN_KFAC: models/curvatures.py KFAC + the sampling_free/ Kronecker
predictive-variance contraction).

    from bnn_kfac_amd.curvatures import KFAC
    kfac = KFAC(net)                      # hooks, like models/curvatures.py:295-317
    ... forward / backward ...; kfac.update(batch_size=B)
    kfac.invert(std ** 2, N)              # inv_state[layer] = (L_A, L_G)

All arithmetic runs in libkfac_hip.so (hand-written gfx950 HIP); there is no CPU
fallback.
"""
from .curvatures import KFAC, Curvature  # noqa: F401

__version__ = "0.1.0"
