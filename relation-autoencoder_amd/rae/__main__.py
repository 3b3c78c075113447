"""python -m rae ...  (the OieInduction.py command line, rae/cli.py)"""
from .cli import main

main()
