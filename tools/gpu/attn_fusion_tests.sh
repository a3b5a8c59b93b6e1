#!/bin/bash
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_qattn.py tests/test_xattn.py 2>&1 | tail -3
