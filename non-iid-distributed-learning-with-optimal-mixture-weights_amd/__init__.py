"""fedamw_amd -- MI355X-native federated round for Non-IID Distributed Learning with
Optimal Mixture Weights (FedAvg / FedProx / FedAMW).

The drop-ins live in ``fedamw_amd.functions.tools`` with the reference's names and
positional signatures (/root/reference/functions/tools.py:329, 356, 413).  All
arithmetic of the round runs in the gfx950 HIP kernels of ``libfedsim.so``
(C-ABI: include/fedsim.h); there is no CPU fallback.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, 'libfedsim.so')

__all__ = ['PKG_DIR', 'LIB_PATH']
