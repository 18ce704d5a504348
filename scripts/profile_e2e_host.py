"""Host-side profile (cProfile) of the end-to-end frame loop (bench.end_to_end
at C3): where the Python time per DPVO.__call__ goes."""
import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import bench  # noqa: E402


def main():
    cfgd = bench.CONFIGS["C3"]
    bench.end_to_end(cfgd, cfgd["buffer"], cfgd["iterations"], 8, warmup=4)   # warm
    pr = cProfile.Profile()
    pr.enable()
    r = bench.end_to_end(cfgd, cfgd["buffer"], cfgd["iterations"], 30, warmup=4)
    pr.disable()
    print(r)
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(45)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
