"""Run a reference script (e.g. code/run_styledmnist_downstream_expr.py) against this package's src/.

    python clear-vae_amd/cvhip/launch.py /path/to/code/run_x.py [script args...]

Direct execution would put the script's directory first on sys.path, so `import src` would resolve to the
reference's package. This launcher puts clear-vae_amd/ first and the script's directory second (so the script's
other local modules still import), then runs the script as __main__ in this process.
"""

import os
import runpy
import sys


def main():
    if len(sys.argv) < 2:
        raise SystemExit(__doc__)
    script = os.path.abspath(sys.argv[1])
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:] = [pkg, os.path.dirname(script)] + [p for p in sys.path[1:] if p not in (pkg,)]
    sys.argv = [script] + sys.argv[2:]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
