"""CLI with the reference's flags (FoodRec/runner.py:16-28):
    python -m FoodRec.runner --model CIKM_Model --dataset Allrecipes [--mg]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from FoodRec.utils.quick_start import quick_start  # noqa: E402


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--model", "-m", type=str, default="SCHGN", help="name of models")
    parser.add_argument("--dataset", "-d", type=str, default="Foodcom", help="Allrecipes or Foodcom")
    parser.add_argument("--mg", action="store_true", help="use Mirror Gradient")
    args, _ = parser.parse_known_args(argv)
    quick_start(model=args.model, dataset=args.dataset, config_dict={"gpu_id": 0}, save_model=True, mg=args.mg)


if __name__ == "__main__":
    main()
