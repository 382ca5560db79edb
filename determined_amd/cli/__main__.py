import sys

from determined_amd.cli import main

sys.exit(main())
