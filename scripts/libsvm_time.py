"""Timing: the native LIBSVM reader vs scikit-learn's load_svmlight_file (+ toarray/float32,
as the reference's loader ends) on a covtype-shaped file.  python scripts/libsvm_time.py [rows]"""
import os
import sys
import tempfile
import time

import numpy as np
from sklearn.datasets import dump_svmlight_file, load_svmlight_file

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd.functions import utils  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 464810
rs = np.random.RandomState(0)
X = np.zeros((n, 54))
X[:, :10] = np.round(rs.rand(n, 10) * 4000)            # covtype's integer-valued quantitative columns
X[np.arange(n), 10 + rs.randint(0, 4, n)] = 1.0
X[np.arange(n), 14 + rs.randint(0, 40, n)] = 1.0
y = rs.randint(1, 8, n)
with tempfile.TemporaryDirectory() as d:
    p = os.path.join(d, 'covtype')
    dump_svmlight_file(X, y, p, zero_based=False)
    mb = os.path.getsize(p) / 1e6
    t0 = time.perf_counter()
    Xs, ys = load_svmlight_file(p)
    Xs = Xs.toarray().astype(np.float32)
    t1 = time.perf_counter()
    Xn, yn, _, _ = utils.read_libsvm(p)
    t2 = time.perf_counter()
    assert np.array_equal(Xn, Xs) and np.array_equal(yn, ys)
    print('%d rows, %.0f MB: sklearn %.2f s, native %.3f s (%d host threads), identical float32 rows'
          % (n, mb, t1 - t0, t2 - t1, min(16, os.cpu_count())))
