import sys

from .dev_client import main

sys.exit(main())
