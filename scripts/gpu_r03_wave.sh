# The north_star wave-per-pair form: parity (oracle cases, fuzz, full-size form equality), then the A/B.
set -o pipefail
mkdir -p gpurun_out/wave
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wave/parity.log 2>&1 && echo PARITY_OK &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_forms.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/wave/forms.log 2>&1 && echo FORMS_OK &&
timeout -k 10 300 python -u scripts/wave_form_ab.py > gpurun_out/wave/ab.jsonl 2> gpurun_out/wave/ab.err && echo AB_OK
