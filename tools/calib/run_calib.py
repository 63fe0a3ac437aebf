"""Drive tools/calib/fetch_calib.so (built by tools/calib/build.sh) under rocprofv3 --pmc."""
import ctypes, os, sys
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "fetch_calib.so"))
N, rows = int(sys.argv[1]) if len(sys.argv) > 1 else 4096 * 16, int(sys.argv[2]) if len(sys.argv) > 2 else 84
assert lib.calib_run(N, rows) == 0
print("known bytes per kernel", N * rows * 4)
