"""Host-side profile of one bench run: python scripts/pyprof_bench.py OUT.txt <bench args...>
(cProfile of bench.main; blocking device syncs show up as the time of the call that waited)."""
import cProfile
import pstats
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

out = sys.argv[1]
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402

pr = cProfile.Profile()
pr.enable()
try:
    bench.main()
finally:
    pr.disable()
    with open(out, "w") as f:
        st = pstats.Stats(pr, stream=f)
        st.sort_stats("cumulative").print_stats(60)
        st.sort_stats("tottime").print_stats(40)
