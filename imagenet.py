"""Drop-in entry point with the reference's command line.

The reference is launched as ``srun python ./imagenet.py --backend=nccl``
(``/root/reference/imagenet.sh:26``) and accepts ``--seed --backend
--batch-size --epochs --lr --save-model`` (``imagenet.py:433-452``). This
script accepts the same flags with the same defaults (plus the extensions in
``imagent_amd/cli.py``) and runs the MI355X-native trainer.
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from imagent_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
