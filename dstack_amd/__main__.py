import sys

from dstack_amd.cli.main import main

sys.exit(main())
