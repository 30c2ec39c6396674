import sys

from .cli import main

if __name__ == "__main__":  # not when a spawned worker imports it
    sys.exit(main())
