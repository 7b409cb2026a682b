timeout -k 10 120 python -u tools/debug/gg_fm.py
