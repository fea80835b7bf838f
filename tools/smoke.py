"""Run __graft_entry__.smoke() on the GPU box (no build step)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
__import__("__graft_entry__").smoke()
