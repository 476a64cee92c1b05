#!/usr/bin/env python3
"""Run the exp.py-counterpart experiment on MI355X (see fedamw_amd/experiment.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import fedamw_amd  # noqa: E402,F401
from fedamw_amd import experiment  # noqa: E402

if __name__ == '__main__':
    experiment.main()
