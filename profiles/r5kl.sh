#!/bin/bash
set -o pipefail
bash profiles/r5l_mfma4.sh && bash profiles/r5k_dog.sh
