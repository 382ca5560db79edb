import sys

from determined_amd.pytorch.dsat._run import main

sys.exit(main())
