# Convenience targets.  `make build` = __graft_entry__.build(); the test_data targets mirror the
# reference's own regression targets (test_data/Makefile) on the data that exists here
# (scripts/test_data_targets.py; EVAL=gpu runs them through the HIP scan instead of the CPU oracle).
PY ?= python
EVAL ?= oracle
GPUFLAG = $(if $(filter gpu,$(EVAL)),--gpu,)

.PHONY: build unit_test cdr1as_test rerun_test test_data test gpu_test

build:
	$(PY) -c "import __graft_entry__ as g; g.build()"

unit_test: build
	$(PY) scripts/test_data_targets.py unit_test $(GPUFLAG)

cdr1as_test: build
	$(PY) scripts/test_data_targets.py cdr1as_test $(GPUFLAG)

rerun_test: build
	$(PY) scripts/test_data_targets.py rerun_test $(GPUFLAG)

test_data: unit_test cdr1as_test rerun_test

test: build
	$(PY) -m pytest tests -x -q -m "not gpu"

gpu_test: build
	$(PY) -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
