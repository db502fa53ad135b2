"""``python -m rdfind_amd [RDFind flags] input.nt ...``"""
import sys

from .program import main

sys.exit(main())
