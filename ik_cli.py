"""`python ik_cli.py --inverse-kine --method {ann,fabrik} --points P.csv ...` --
the reference's CLI entry point (cli.py:382-388) for the MI355X engine."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from inversekinematicsann_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
