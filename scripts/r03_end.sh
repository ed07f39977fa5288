#!/bin/bash
# end-of-round set: -m gpu suite + smoke + bench line, then the rocprof kernel
# table, PMC traffic of the decoder and a second bench line
set -o pipefail
bash scripts/r03_final.sh e3 && bash scripts/r03_measure.sh
