#!/usr/bin/env python3
"""OpenAI-compatible server (see lumen/cli/serve.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lumen.cli.serve import main  # noqa: E402

if __name__ == "__main__":
    main()
