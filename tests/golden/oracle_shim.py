"""Import shim so gen_golden.py (run with cwd=/root/reference) can reach the build's oracle.
Used only to produce codewords for the golden inputs; every expected OUTPUT comes from the
reference itself."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle.ldpc_oracle import *  # noqa: E402,F401,F403
from oracle.ldpc_oracle import encode  # noqa: E402,F401
