timeout -k 10 120 python tests/diag_kin.py
