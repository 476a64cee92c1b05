"""Per-dataset hyper-parameters -- drop-in for the reference's ``get_parameter``
(/root/reference/functions/optimal_parameters.py:1-165, used at exp.py:41-53 and tune.py).

A table instead of an if-chain: each named dataset maps to its tuned values; anything
else gets the reference's fall-through branch (optimal_parameters.py:153-163), which --
as in the reference -- has no ``lr_p`` / ``lr_p_os`` / ``lambda_reg_os`` keys (a9a and
covtype land there; the exp driver states the values it picks for them).  Every dict
also carries ``local_update = 100`` (optimal_parameters.py:164).
"""

_KEYS = ('task_type', 'num_examples', 'dimensional', 'num_classes', 'kernel_type', 'kernel_par',
         'lambda_reg_os', 'lambda_reg', 'lambda_prox', 'alpha_Dirk', 'lr', 'lr_p_os', 'lr_p')

# dataset: (n_examples, d, classes, sigma, lambda_reg_os, lambda_reg, lambda_prox, lr_p_os, lr_p)
# -- classification datasets with the full key set (alpha_Dirk 0.01, lr 0.5, gaussian kernel)
_TUNED = {
    'mnist': (60000, 784, 10, 0.1, 5e-6, 5e-6, 1e-6, 1e-3, 1e-3),
    'dna': (2000, 180, 3, 0.1, 1e-6, 1e-2, 1e-2, 0.1, 1e-3),
    'letter': (15000, 16, 26, 0.1, 5e-5, 5e-3, 5e-5, 1e-3, 1e-4),
    'pendigits': (7494, 16, 10, 0.01, 5e-3, 1e-2, 1e-3, 0.5, 5e-4),
    'satimage': (4435, 36, 6, 0.1, 1e-3, 1e-3, 5e-4, 0.1, 1e-5),
    'usps': (7291, 256, 10, 0.1, 5e-4, 5e-5, 1e-4, 5e-3, 5e-4),
}

# datasets whose entry is the reference's default block under their own name (poker,
# Sensorless, shuttle: optimal_parameters.py), and the regression toy problem
_DEFAULT = dict(task_type='classification', num_classes=10, dimensional=784, kernel_type='gaussian',
                kernel_par=0.1, lambda_reg=1e-5, lambda_prox=7e-7, lr=0.001)
_SYNTHETIC_NONLINEAR = dict(task_type='regression', num_examples=10000, dimensional=10, num_classes=1,
                            kernel_type='gaussian', kernel_par=0.1, lambda_reg=1e-6, lambda_prox=7e-7,
                            alpha_Dirk=1, lr=0.001)


def get_parameter(dataset):
    """Hyper-parameter dict for ``dataset`` (same keys, values and key order as the reference)."""
    if dataset in _TUNED:
        n, d, C, sig, lam_os, lam, prox, lrp_os, lrp = _TUNED[dataset]
        vals = ('classification', n, d, C, 'gaussian', sig, lam_os, lam, prox, 0.01, 0.5, lrp_os, lrp)
        out = dict(zip(_KEYS, vals))
    elif dataset == 'synthetic_nonlinear':
        out = dict(_SYNTHETIC_NONLINEAR)
    else:
        out = dict(_DEFAULT)
    out['local_update'] = 100
    return out
