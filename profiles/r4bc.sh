#!/bin/bash
set -o pipefail
bash profiles/r4b_check.sh && bash profiles/r4c_dog.sh && bash profiles/r4d_split.sh && bash profiles/r4e_env.sh
