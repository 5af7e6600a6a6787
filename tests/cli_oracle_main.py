"""``python tests/cli_oracle_main.py <cli args>``: the CLI with the CPU oracle as the breakpoint
search, as a process of its own, so tests can feed it a real stdin pipe (find_circ.py:467-469)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.dirname(HERE), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

from find_circ2_amd import cli  # noqa: E402
from oracle_engine import oracle_evaluator_factory  # noqa: E402

if __name__ == "__main__":
    sys.exit(cli.main(sys.argv[1:], evaluator_factory=oracle_evaluator_factory))
