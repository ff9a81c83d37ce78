"""Host-side (Python) profile of one training step: where the CPU time goes when a step is
launch-bound.   python tools/host_profile.py [pretrain|finetune] [B]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "pretrain"
    B = sys.argv[2] if len(sys.argv) > 2 else "4"
    mod = __import__(f"tools.{'pretrain_bench' if which == 'pretrain' else 'train_bench'}", fromlist=["main"])
    sys.argv = [sys.argv[0], "--batch", B, "--steps", os.environ.get("HP_STEPS", "2"), "--warmup", "1"]
    pr = cProfile.Profile()
    pr.enable()
    mod.main()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
