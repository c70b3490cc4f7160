#!/bin/bash
timeout -k 10 300 python tools/bench_gemm_layouts.py
