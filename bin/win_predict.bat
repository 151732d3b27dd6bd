@echo off
rem Windows batch prediction (reference: bin/win_predict.bat).
rem usage: bin\win_predict.bat MODEL FILE_OR_DIR [CONF] [SAVE_MODE] [PREDICT_TYPE] [EVAL_METRICS]
set MODEL=%1
set FILE=%2
set CONF=%3
if "%CONF%"=="" set CONF=config\model\%MODEL%.conf
set MODE=%4
if "%MODE%"=="" set MODE=PREDICT_RESULT_ONLY
set PTYPE=%5
if "%PTYPE%"=="" set PTYPE=value
set METRICS=%6
if "%METRICS%"=="" set METRICS=auc,mae
if not exist log mkdir log
python -m ytk_learn_amd.cli.predict %CONF% %MODEL% %FILE% false "" %MODE% _%MODEL%_%MODE% 100 %METRICS% %PTYPE%
