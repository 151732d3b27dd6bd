@echo off
rem Windows launcher (reference: bin/win_local_optimizer.bat). CPU or a single device.
rem usage: bin\win_local_optimizer.bat MODEL [CONF] [TRANSFORM_SCRIPT]
set MODEL=%1
set CONF=%2
if "%CONF%"=="" set CONF=config\model\%MODEL%.conf
if not exist log mkdir log
if "%3"=="" (
  python -m ytk_learn_amd.cli.train %MODEL% %CONF%
) else (
  python -m ytk_learn_amd.cli.train %MODEL% %CONF% --transform-script %3
)
