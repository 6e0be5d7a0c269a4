"""Run bench.py against an alternative build of the library (dev A/B tool):
python tools/bench_with_lib.py <path/to/libmmla_variant.so> [bench.py args...]"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mmla_audio_amd import _lib  # noqa: E402

_lib.load_library(sys.argv[1])
sys.argv = [os.path.join(REPO, 'bench.py')] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name='__main__')
