"""ncf_amd -- MI355X-native NeuMF training hot path (drop-in for YonkaMayonkaZ/NCF).

Native code: ``libncf_hip.so`` (HIP kernels for gfx950, C ABI in include/ncf_hip.h)
and ``libncf_sampler.so`` (host negative sampler, include/ncf_sampler.h), both
built in-tree by ``make -C ncf_amd/csrc``.
"""
__version__ = "0.1.0"
