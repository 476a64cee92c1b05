"""Package surface (CPU): every module imports and exposes the drop-in API."""
import inspect

import fedamw_amd
from fedamw_amd import data, dist, engine, rng
from fedamw_amd.functions import tools


def test_engine_classes():
    for name in ('Features', 'Shuffler', 'LocalTrainer', 'Aggregator', 'Evaluator', 'Mixture', 'pad_ld'):
        assert hasattr(engine, name), name


def test_dropin_signatures_match_reference_order():
    """Positional parameter order of the reference (tools.py:329, 356, 413)."""
    fed = ['X_train', 'y_train', 'X_test', 'y_test', 'type', 'num_classes', 'D', 'lr', 'epoch', 'batch_size',
           'prox', 'mu', 'lambda_reg_if', 'lambda_reg', 'round']
    for fn in (tools.FedAvg, tools.FedProx):
        ps = [p.name for p in inspect.signature(fn).parameters.values() if p.kind == p.POSITIONAL_OR_KEYWORD]
        assert ps == fed
    ps = [p.name for p in inspect.signature(tools.FedAMW).parameters.values() if p.kind == p.POSITIONAL_OR_KEYWORD]
    assert ps == fed[:4] + ['validloader'] + fed[4:] + ['lr_p']
    assert inspect.signature(tools.FedProx).parameters['prox'].default is True
    assert inspect.signature(tools.FedAMW).parameters['lambda_reg_if'].default is True


def test_no_cpu_fallback():
    import torch
    import pytest
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(RuntimeError):
        tools.FedAvg([torch.zeros(4, 8)], [torch.zeros(4, dtype=torch.long)], torch.zeros(2, 8),
                     torch.zeros(2, dtype=torch.long), 'classification', 2, 8, round=1)


def test_lr_schedule_matches_reference_semantics():
    lr, seq = 0.5, []
    for t in range(8):
        lr = tools.update_learning_rate(t, lr, 8)
        seq.append(lr)
    assert seq[:4] == [0.5] * 4 and abs(seq[4] - 0.05) < 1e-15 and abs(seq[6] - 0.0005) < 1e-15
