# interleaved contraction + staged row stores (bins_ilv) vs the prefetch form, across segments-per-wave
set -o pipefail
cd scripts || exit 1
SETTINGS="bins_ilv=0;bins_ilv=1;bins_ilv=0;bins_ilv=1;bins_ilv=1,demod_spw=3;bins_ilv=1,demod_spw=4;bins_ilv=1,demod_spw=1" timeout -k 10 300 python tune_rows_demod.py || exit 1
NSEG=1250000 SETTINGS="bins_ilv=0;bins_ilv=1;bins_ilv=1,demod_spw=4;bins_ilv=1,demod_spw=8" timeout -k 10 300 python tune_rows_demod.py || exit 1
SETTINGS="bins_ilv=0;bins_ilv=1;bins_ilv=0;bins_ilv=1;bins_ilv=1,demod_spw=3;bins_ilv=1,demod_spw=4" timeout -k 10 300 python tune_step.py || exit 1
