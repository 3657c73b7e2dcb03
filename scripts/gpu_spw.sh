# segments-per-wave sweep: roofline kernel (100k and 1.25M segments) and the whole step
set -o pipefail
cd scripts || exit 1
SETTINGS="demod_spw=0;demod_spw=1;demod_spw=2;demod_spw=3;demod_spw=4" timeout -k 10 300 python tune_rows_demod.py || exit 1
NSEG=1250000 SETTINGS="demod_spw=0;demod_spw=2;demod_spw=4;demod_spw=8;demod_spw=16" timeout -k 10 300 python tune_rows_demod.py || exit 1
SETTINGS="demod_spw=0;demod_spw=1;demod_spw=2;demod_spw=3" timeout -k 10 300 python tune_step.py || exit 1
