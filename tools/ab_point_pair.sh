for v in base ppall base ppall; do STL_LIB_PATH=build/ab/$v.so timeout -k 10 120 python -u tools/perf_variant.py || exit 1; done
