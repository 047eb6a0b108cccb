"""GPU pytest run against a given libicap build (a variant from tools/build_variant.py).
usage: python tools/libtest.py LIB.so PYTEST_ARGS..."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from image_caption_amd import _lib

_lib.load(sys.argv[1])
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[2:] + ["-m", "gpu", "-x", "-q", "-p", "no:cacheprovider", "--timeout", "200",
                                     "--timeout-method", "thread"]))
