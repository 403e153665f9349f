"""hb_mcmc_amd -- MI355X (gfx950) implementation of the sidruns30/HB_MCMC
heartbeat-binary light-curve log-likelihood path.

* ``libhbmi.so`` (hb_mcmc_amd/csrc, C-ABI in include/hbmi.h): HIP kernels +
  the likelihood3.h drop-in symbols + a batched context API.
* ``hb_mcmc_amd.likelihood``: Python mirror of the batched API (ctypes).
* ``hb_mcmc_amd.pyHB``: drop-in for the reference Cython module ``pyHB``.
* ``hb_mcmc_amd.sampler``: the parallel-tempered MCMC caller (mcmc_wrapper2.c).
* ``hb_mcmc_amd.dist``: temperature slots sharded over GPUs with an RCCL all-gather.
* ``hb_mcmc_amd.catalog``: catalog-sweep mode (many targets per GPU, every
  size class in one eval launch; targets dealt over GPUs).

Importing the package does not touch the GPU.
"""
__version__ = "0.1.0"

from ._lib import HBMIError  # noqa: E402,F401
