@echo off
rem Windows LibSVM -> ytk-learn converter (reference: bin/win_libsvm_convert_2_ytklearn.bat).
rem usage: bin\win_libsvm_convert_2_ytklearn.bat MODE IN OUT
python -m ytk_learn_amd.tools.libsvm_convert %1 "###" "," "," ":" local %2 %3
