#!/usr/bin/env python3
"""CLI shim: ``python bench/prof_summary.py <rocprofv3 dir>`` -> markdown (kgs.utils.profile)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kgs.utils.profile import main  # noqa: E402

if __name__ == "__main__":
    main()
