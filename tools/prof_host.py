"""Host-side (Python) profile of a bench run: python tools/prof_host.py <bench args...>.
Prints the functions with the largest self time (cProfile)."""
import cProfile
import pstats
import runpy
import sys

sys.argv = ["bench.py"] + sys.argv[1:]
pr = cProfile.Profile()
pr.enable()
try:
    runpy.run_path("bench.py", run_name="__main__")
finally:
    pr.disable()
    st = pstats.Stats(pr, stream=sys.stderr)
    st.sort_stats("tottime").print_stats(40)
    st.sort_stats("cumulative").print_stats("ytk_learn_amd", 40)
